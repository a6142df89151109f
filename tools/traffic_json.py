"""Per-launch HBM traffic of the roofline GEMM from the FETCH_SIZE / WRITE_SIZE
rocprofv3 passes of tools/pmc_gemm.sh, corrected as MI355X_MICROARCH.md
(HBM) prescribes: gfx950 FETCH_SIZE counts half of the bytes of 16-B/lane
streaming reads (reads = 2 x FETCH_SIZE); WRITE_SIZE is exact for 16-B/lane
stores.  Counter units are KB.  The first launch (cold caches, code load) is
dropped; a launch = every GEMM dispatch of that ops.gemm call."""
import csv
import json
import os
import statistics
import sys

d = sys.argv[1]
# optional: which kernel (name substring) and its algorithmic bytes per launch
KSUB = sys.argv[2] if len(sys.argv) > 2 else "gemm"


def per_dispatch(sub, counter):
    path = os.path.join(d, sub, "run_counter_collection.csv")
    vals = []
    for r in csv.DictReader(open(path)):
        if KSUB in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"]))
    vals.sort()
    return vals


f = per_dispatch("fetch", "FETCH_SIZE")
w = per_dispatch("write", "WRITE_SIZE")
fk = [v for _, v, _ in f][1:]
wk = [v for _, v, _ in w][1:]
if len(sys.argv) > 5:   # only the last N dispatches of that kernel (a probe's timed launches)
    nlast = int(sys.argv[5])
    fk, wk = fk[-nlast:], wk[-nlast:]
M, N, K = 10688, 1024, 16448
alg = int(sys.argv[3]) if len(sys.argv) > 3 else 4 * (M * K + N * K + M * N)
probe = sys.argv[4] if len(sys.argv) > 4 else "tools/pmc_gemm.sh over tools/roofline_probe.py"
hbm = 2 * 1024 * statistics.mean(fk) + 1024 * statistics.mean(wk)
print(json.dumps({
    "kernel": f[0][2].split("(")[0] if f else None,
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
              f"{probe} (5 launches, first dropped)",
    "FETCH_SIZE_KB_mean": statistics.mean(fk), "WRITE_SIZE_KB_mean": statistics.mean(wk),
    "correction": "gfx950 FETCH_SIZE counts 1/2 of wide (16 B/lane) streaming reads "
                  "(MI355X_MICROARCH.md HBM): reads = 2*FETCH_SIZE; WRITE_SIZE exact",
    "hbm_bytes_per_launch": int(hbm),
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": round(hbm / alg, 2),
}, indent=1))
