"""Per-stream busy time, GPU-busy union and idle gaps of one step window in a
rocprofv3 kernel trace.  usage: stream_timeline.py <prof_dir> [optimizer launches per step]
The window ends at the last 'k_adam_many' launch and starts after the one
that many launches earlier (C3: 1 per step, C5: 2)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_many" in r["Kernel_Name"]]
# step window = between the last two optimizer launches
per = int(sys.argv[2]) if len(sys.argv) > 2 else 1
i0, i1 = adam[-1 - per] + 1, adam[-1] + 1
win = rows[i0:i1]
t0 = int(win[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in win)
print(f"step window: {len(win)} kernels, {(t1 - t0) / 1e3:.1f} us")
busy = collections.defaultdict(int)
names = collections.defaultdict(lambda: collections.defaultdict(int))
for r in win:
    dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy[r["Stream_Id"]] += dur
    names[r["Stream_Id"]][r["Kernel_Name"][:50]] += dur
for s, b in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f"stream {s}: busy {b / 1e3:.1f} us, {sum(1 for r in win if r['Stream_Id'] == s)} kernels")
    for n, v in sorted(names[s].items(), key=lambda kv: -kv[1])[:6]:
        print(f"    {v / 1e3:8.1f}  {n}")
# union of busy intervals and gaps
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win)
union, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s, e in iv[1:]:
    if s > cur_e:
        union += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
print(f"GPU busy (union): {union / 1e3:.1f} us; idle gaps: {len(gaps)} totalling {sum(gaps) / 1e3:.1f} us, "
      f"largest {sorted(gaps)[-5:] if gaps else []} ns")
