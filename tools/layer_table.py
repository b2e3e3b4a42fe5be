"""Per-(kernel, grid) timing table from a rocprofv3 kernel trace. usage: layer_table.py <prof_dir> <steps>"""
import collections
import csv
import glob
import os
import sys

d, steps = sys.argv[1], int(sys.argv[2])
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
g = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    nm = r["Kernel_Name"]
    if "sel::" not in nm and "_ZN3sel" not in nm:
        continue
    for tag in ("k_conv_fwd_bf16", "k_conv_fwd", "k_wgrad_bf16", "k_conv_wgrad", "k_split_sum", "k_rvq_fwd",
                "k_logmel", "k_pack", "k_unpack", "k_replicate"):
        if tag in nm:
            break
    else:
        tag = nm[:30]
    if "Li" in nm and "k_conv_fwd" in nm:
        tag += nm[nm.find("ILi"):nm.find("ILi") + 14]
    elif "<" in nm:
        tag += nm[nm.find("<"):nm.find("<") + 10]
    key = (tag, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"],
           r["LDS_Block_Size"], r["VGPR_Count"])
    g[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = 0
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:40]:
    tot += sum(v)
    print(f"{sum(v) / steps / 1e3:8.1f} us/step n/step={len(v) / steps:4.1f} avg={sum(v) / len(v) / 1e3:8.1f}us {k}")
