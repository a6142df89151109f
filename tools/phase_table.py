#!/usr/bin/env python3
"""Per-phase kernel time from a rocprofv3 run with roctx ranges (ainp.trace:
AINP_TRACE=1 puts data / fwd / bwd / allreduce / optimizer ranges around each
training-step phase):

  AINP_TRACE=1 rocprofv3 --marker-trace --hip-runtime-trace --kernel-trace \\
      -f csv -d <dir> -o run -- python3 bench.py --steps 5 --warmup 2 ...
  python3 tools/phase_table.py <dir>

Each kernel dispatch is attributed to the innermost range that was open
(on any thread: autograd's engine thread launches the backward while the
main thread sits in its "bwd" range) when its HIP launch call ran (kernel Correlation_Id ->
HIP API row -> host timestamp -> marker ranges).  Prints, per phase, the
number of dispatches, the summed kernel time and its share, and per-phase
top kernels; kernels launched outside every range go to "(none)"."""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def _rows(d, suffix):
    fs = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    out = []
    for f in fs:
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def ranges(markers):
    """[(thread, start, end, name)] from the marker API trace (push/pop pairs
    are reported as one row with Start/End timestamps and the message)."""
    rs = []
    for r in markers:
        name = r.get("Message") or r.get("Function") or ""
        fn = r.get("Function", "")
        if fn and "RangePop" in fn:
            continue
        try:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        except (KeyError, ValueError):
            continue
        if e <= s:
            continue
        rs.append((r.get("Thread_Id"), s, e, name))
    return rs


def main(d):
    kern = _rows(d, "kernel_trace.csv")
    api = _rows(d, "hip_api_trace.csv")
    mk = _rows(d, "marker_api_trace.csv")
    if not kern:
        sys.exit(f"no kernel_trace.csv under {d}")
    launch = {}
    for r in api:
        launch[r["Correlation_Id"]] = (r.get("Thread_Id"), int(r["Start_Timestamp"]))
    rs = ranges(mk)
    tot = collections.Counter()
    cnt = collections.Counter()
    top = collections.defaultdict(collections.Counter)
    for k in kern:
        dur = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3   # us
        ph = "(none)"
        li = launch.get(k["Correlation_Id"])
        if li is not None:
            th, t = li
            best = None
            for (rth, s, e, nm) in rs:
                # time containment only: the backward's kernels are launched by
                # autograd's engine thread while the main thread sits in "bwd"
                if s <= t <= e:
                    if best is None or (e - s) < best[0]:
                        best = (e - s, nm)
            if best:
                ph = best[1]
        tot[ph] += dur
        cnt[ph] += 1
        top[ph][k["Kernel_Name"][:70]] += dur
    allt = sum(tot.values())
    print(f"{'phase':<12} {'dispatches':>10} {'kernel ms':>10} {'share':>7}")
    for ph, t in tot.most_common():
        print(f"{ph:<12} {cnt[ph]:>10} {t / 1e3:>10.3f} {t / allt:>7.3f}")
    for ph, _ in tot.most_common():
        print(f"\n[{ph}] top kernels (ms)")
        for kn, t in top[ph].most_common(6):
            print(f"  {t / 1e3:9.3f}  {kn}")


if __name__ == "__main__":
    main(sys.argv[1])
