#!/usr/bin/env python3
"""Step timeline from a rocprofv3 kernel_trace.csv: splits the trace at each
stft512/stft_features launch (one per train step), and per step reports wall
(first start .. next step's first start), busy (union of kernel intervals),
idle gaps and the per-kernel union time.  tools/timeline.py <trace.csv> [step]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
              r["Stream_Id"]) for r in rows), key=lambda x: x[0])
starts = [i for i, k in enumerate(ks) if "stft512" in k[2] or "stft_features" in k[2]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) - 2
a, b = starts[which], starts[which + 1]
seg = ks[a:b]
t0, t1 = seg[0][0], ks[b][0]
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e, n, st in seg:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"step {which}: wall {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, "
      f"{len(seg)} kernels, idle {(t1 - t0 - busy) / 1e6:.3f} ms in {len(gaps)} gaps")
gaps.sort(reverse=True)
for g, n in gaps[:12]:
    print(f"  gap {g / 1e3:8.1f} us before {n[:90]}")
tot = defaultdict(int)
for s, e, n, st in seg:
    tot[n[:80]] += e - s
print("  kernel time (may overlap across streams):")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:25]:
    print(f"  {t / 1e6:7.3f} ms  {n}")
