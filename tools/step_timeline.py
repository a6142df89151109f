"""Timeline of one training step from a rocprofv3 --kernel-trace CSV: every
dispatch of the step (start offset, duration, stream) and, for the critical
(main) stream, the idle gaps between its kernels -- what the step time is
made of once side-stream overlap is accounted for.

  python tools/step_timeline.py run_kernel_trace.csv [step_marker_kernel] [which]

A step starts at each dispatch whose name contains step_marker_kernel
(default: stft512_kernel); `which` picks the step (default: -2, the last
complete one)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "stft512_kernel"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(starts) < 2:
    sys.exit("fewer than two step markers")
a = starts[which]
b = starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
t_end = max(int(r["End_Timestamp"]) for r in step)
print(f"step span {(int(step[-1]['Start_Timestamp']) - t0) / 1e6:.3f} ms to last start, "
      f"{(t_end - t0) / 1e6:.3f} ms to last end, {len(step)} dispatches")
queues = sorted({r["Queue_Id"] for r in step})
busy = {}
for q in queues:
    ks = [r for r in step if r["Queue_Id"] == q]
    busy[q] = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks)
    print(f"queue {q}: {len(ks)} dispatches, busy {busy[q] / 1e6:.3f} ms")
main = max(queues, key=lambda q: sum(1 for r in step if r["Queue_Id"] == q))
print(f"\n(main queue = {main})  t_start(ms)  dur(ms)  gap_before(ms)  queue  kernel")
prev_end = {}
gap_total = 0
for r in step:
    s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
    gap = (s - prev_end[q]) if q in prev_end else 0
    if q == main:
        gap_total += max(gap, 0)
    prev_end[q] = max(e, prev_end.get(q, 0))
    name = r["Kernel_Name"].replace("void ", "").replace("ainp::", "")[:70]
    print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} {gap / 1e6:8.3f}  {q:>3}  {name}")
print(f"\nmain-queue idle gaps in the step: {gap_total / 1e6:.3f} ms")
