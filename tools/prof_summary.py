"""Summarise a rocprofv3 kernel-trace database (rocpd .db) into the tracked
profiles/ files.

  python tools/prof_summary.py <results.db> <steps> <out_prefix>

writes <out_prefix>_kernel_stats.csv (per kernel: calls, total/avg ns, ms per
step over <steps> profiled steps incl. warmup) and <out_prefix>_roofline_kernel.json
(the bench's roofline kernel = the LSTM layer-0 input-projection GEMM,
selected by name + grid (336 tiles x 256 threads, 2 pointer batches = the
two directions); layers 1/2 launch the same grid with K=256 instead of
16448, i.e. 1/64 of the work, and are excluded by duration).
"""
import csv
import json
import sqlite3
import sys
from collections import defaultdict

db, steps, prefix = sys.argv[1], int(sys.argv[2]), sys.argv[3]
c = sqlite3.connect(db)
rows = list(c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels"))
agg = defaultdict(lambda: [0, 0])
for name, dur, *_ in rows:
    agg[name][0] += 1
    agg[name][1] += dur
total = sum(v[1] for v in agg.values())
with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MsPerStep"])
    for name, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([name, n, d, round(d / n, 1), round(100.0 * d / total, 3),
                    round(d / 1e6 / steps, 4)])
# Since the stream-K GEMM, the L0 forward projection (672 tiles of 128x128 on
# 768 resident slots) is the stream-K kernel (768 x 256 threads) + its fixup
# (one block per tile: 672 x 256); older builds launched the plain grid
# (336 x 256, 2).  The K=256 layers 1/2 use the plain grid at 1/64 of the work
# and are excluded by duration.
sk = [dur for name, dur, gx, gy, gz, wx in rows
      if name.startswith("void ainp::gemm_f32_streamk<")
      and name.split(">")[0].endswith("true, true, true, true") and gx == 768 * 256]
fix = [dur for name, dur, gx, gy, gz, wx in rows
       if name.startswith("ainp::gemm_streamk_fixup") and gx == 672 * 256]
# plain grid: gemm_f32_kernel<true, true, true, true> (exact f32, older builds)
# or gemm_f32_kernel<X6, true, true, true, true> (both main loops since the
# three-piece bf16 split)
same = [dur for name, dur, gx, gy, gz, wx in rows
        if (name.startswith("void ainp::gemm_f32_kernel<true, true, true, true>")
            or name.startswith("void ainp::gemm_f32_kernel<true, true, true, true, true>")
            or name.startswith("void ainp::gemm_f32_kernel<false, true, true, true, true>"))
        and gx == 336 * 256 and gy == 2]
if sk:
    l0 = [d for d in sk if d > 0.5 * max(sk)]
    fix_avg = sum(fix) / len(fix) if fix else 0.0
    kname = ("gemm_f32_streamk<true,true,true,true> grid 768x256 + gemm_streamk_fixup 672x256 "
             "(LSTM l0 input projection M=10688 N=1024 K=16448)")
else:
    l0 = [d for d in same if d > 0.2 * max(same)] if same else []
    fix_avg = 0.0
    kname = ("gemm_f32_kernel<X6=true,...> grid (336x256, 2) (LSTM l0 input projection "
             "M=10688 N=1024 K=16448, three-piece bf16 split main loop)")
out = {"kernel": kname,
       "launches": len(l0),
       "avg_ns": round(sum(l0) / max(1, len(l0)) + fix_avg, 1),
       "fixup_avg_ns": round(fix_avg, 1),
       "min_ns": min(l0) if l0 else None, "max_ns": max(l0) if l0 else None,
       "flop_per_launch": 2.0 * 10688 * 1024 * 16448}
if l0:
    out["achieved_tflops_at_avg"] = round(out["flop_per_launch"] / (out["avg_ns"] * 1e-9) / 1e12, 2)
json.dump(out, open(prefix + "_roofline_kernel.json", "w"), indent=1)
print(json.dumps(out))
print("total ms/step (all kernels / steps):", round(total / 1e6 / steps, 3))
for name, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{d/1e6/steps:8.3f} ms/step {n:5d} {d/n/1e3:9.1f} us  {name[:110]}")
