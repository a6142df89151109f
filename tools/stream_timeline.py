#!/usr/bin/env python3
"""One train step of a rocprofv3 kernel_trace.csv as a per-stream listing:
every kernel with its start offset from the step's first launch, duration and
stream, plus a per-stream busy total and the intervals where only one stream
(or none) runs.  Steps are split at the stft512 / stft_features launches.

  tools/stream_timeline.py <kernel_trace.csv> [step] [--min-us 5]
"""
import csv
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    min_us = 5.0
    if "--min-us" in sys.argv:
        min_us = float(sys.argv[sys.argv.index("--min-us") + 1])
        args = [a for a in args if a != str(sys.argv[sys.argv.index("--min-us") + 1])]
    rows = list(csv.DictReader(open(args[0])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                  r["Stream_Id"]) for r in rows), key=lambda x: x[0])
    starts = [i for i, k in enumerate(ks) if "stft512" in k[2] or "stft_features" in k[2]]
    which = int(args[1]) if len(args) > 1 else len(starts) - 2
    a, b = starts[which], starts[which + 1]
    seg = ks[a:b]
    t0, t1 = seg[0][0], ks[b][0]
    streams = sorted({k[3] for k in seg})
    col = {s: i for i, s in enumerate(streams)}
    print(f"step {which}: wall {(t1 - t0) / 1e6:.3f} ms; streams {streams}")
    busy = {s: 0 for s in streams}
    for s, e, n, st in seg:
        busy[st] += e - s
        if (e - s) / 1e3 >= min_us:
            pad = "    " * col[st]
            name = n.replace("void ", "").replace("ainp::", "")[:70]
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {pad}s{col[st]} {name}")
    for st in streams:
        print(f"stream {st}: kernel time {busy[st] / 1e6:.3f} ms")
    # concurrency profile: time with 0, 1, >=2 streams active
    ev = []
    for s, e, n, st in seg:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    act, last = 0, t0
    acc = {0: 0, 1: 0, 2: 0}
    for t, d in ev:
        acc[min(act, 2)] += t - last
        act += d
        last = t
    acc[0] += t1 - last
    print("time with 0 / 1 / >=2 kernels running: "
          + " / ".join(f"{acc[k] / 1e6:.3f}" for k in (0, 1, 2)) + " ms")


if __name__ == "__main__":
    main()
