"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE
cannot share a pass on gfx950: MI355X_MICROARCH.md "rocprofv3 PMC slots").

Corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE (KB) reports 1/2 of the
bytes of 16-B-per-lane streaming reads on gfx950 -> x2; WRITE_SIZE (KB) is exact
for 16-B stores.  Both count Infinity-Cache hits, so sizes must exceed 256 MB
of live data to read them as HBM bytes (C3 per-layer tensors are 100-300 MB).

usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json> [steps | auto]
(steps: training steps in the profiled run -> a per-step total over the sel kernels,
 leaving out the bench's B = 512 STFT roofline probe)
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            k = row["Kernel_Name"]
            acc[k][0] += 1
            acc[k][1] += float(row["Counter_Value"])
    return acc


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in set(fetch) | set(write):
        nf, sf = fetch.get(k, [0, 0.0])
        nw, sw = write.get(k, [0, 0.0])
        if not nf or not nw:
            continue
        fb = 2.0 * 1024.0 * sf / nf  # KB -> B, x2 gfx950 wide-read correction
        wb = 1024.0 * sw / nw
        out[k] = {"launches": nf, "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                  "traffic_bytes_per_launch": round(fb + wb)}
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    if len(sys.argv) > 4:
        # auto: one sel Adam update per step (k_adam_many launches)
        steps = (sum(v["launches"] for k, v in out.items() if "k_adam_many" in k) or 1) if sys.argv[4] == "auto" \
            else int(sys.argv[4])
        tot = sum(v["traffic_bytes_per_launch"] * v["launches"] for k, v in out.items()
                  if ("sel::" in k or "_ZN3sel" in k) and "k_stft_mag_fwd" not in k)
        print(f"sel kernels, all launches except the STFT probe: {tot / 1e9:.2f} GB over {steps} steps = "
              f"**{tot / steps / 1e9:.2f} GB/step**\n")
    top = sorted(out.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"] * kv[1]["launches"])[:25]
    print("| kernel | launches | fetch MB/launch (x2 corr.) | write MB/launch | traffic MB/launch |")
    print("|---|---|---|---|---|")
    for k, v in top:
        print(f"| `{k[:90]}` | {v['launches']} | {v['fetch_bytes_per_launch'] / 1e6:.2f} | "
              f"{v['write_bytes_per_launch'] / 1e6:.2f} | {v['traffic_bytes_per_launch'] / 1e6:.2f} |")


if __name__ == "__main__":
    main()
