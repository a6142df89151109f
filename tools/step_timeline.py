"""Timeline of one training step from a rocprofv3 --kernel-trace CSV: every
dispatch of the step (start offset, duration, stream), the idle gaps of the
critical (main) stream, each stream's busy time, and the main stream's
critical path split into the step's phases -- what the step time is made of
once side-stream overlap is accounted for.

  python tools/step_timeline.py run_kernel_trace.csv [step_marker_kernel] [which]
  python tools/step_timeline.py --extract run_kernel_trace.csv out.csv [which]
      (write that one step's rows: the committed profiles/steps/*_trace.csv
      that bench.py's critical-path table reads)

A step starts at each dispatch whose name contains step_marker_kernel
(default: stft512_kernel); `which` picks the step (default: -2, the last
complete one)."""
import csv
import sys

# CNNBLSTM step phases on the main stream, in order: (name, predicate on a
# kernel name that opens the phase).  "after_last" phases open at the first
# match behind the last dispatch of the previous phase's kernel.
CNN_PHASES = [
    ("features", lambda n: "stft512_kernel" in n or "stft_features" in n),
    ("encoder_fwd", lambda n: "conv3x3" in n),
    ("bridge_l0_projection", lambda n: "bn_relu_apply_ntcf" in n),
    ("blstm_fwd", lambda n: "lstm_fwd_kernel" in n),
    ("decoder_fwd_loss", lambda n: "conv3x3" in n),
    ("decoder_bwd", lambda n: "scale_by_dev" in n),
    ("bptt", lambda n: "lstm_bwd_kernel" in n),
    ("l0_backward", None),          # first main dispatch after the last BPTT's hprev
    ("encoder_bwd", lambda n: "bn_relu_bwd" in n and "ntcf" in n),
    ("optimizer", lambda n: "adam_kernel" in n),
]


def load_step(path, marker="stft512_kernel", which=-2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(starts) < 2 and len(starts) != 1:
        raise SystemExit("no step markers")
    if len(starts) == 1:            # an extracted one-step trace
        return rows[starts[0]:]
    a = starts[which]
    b = starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
    return rows[a:b]


def critical_path(step, phases=CNN_PHASES):
    """Per-stream busy ms and the main stream's critical path per phase (ms
    from the phase's first main-stream dispatch to the next phase's, the last
    one to the step's last end): the phases sum to the step's span."""
    t0 = int(step[0]["Start_Timestamp"])
    t_end = max(int(r["End_Timestamp"]) for r in step)
    queues = sorted({r["Queue_Id"] for r in step})
    busy = {q: sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                   for r in step if r["Queue_Id"] == q) / 1e6 for q in queues}
    main = max(queues, key=lambda q: sum(1 for r in step if r["Queue_Id"] == q))
    ms = [r for r in step if r["Queue_Id"] == main]
    names = [r["Kernel_Name"] for r in ms]
    bounds = [0]
    i = 0
    for k in range(1, len(phases)):
        name, pred = phases[k]
        if pred is None:            # behind the last dispatch of the previous phase's kernel
            prev = phases[k - 1][1]
            last = max((j for j in range(i, len(names)) if prev(names[j])), default=i)
            j = last + 1
            while j < len(names) and ("hprev" in names[j] or "sum_slabs" in names[j]):
                j += 1
        else:
            j = next((j for j in range(i + 1, len(names)) if pred(names[j])), None)
        if j is None or j >= len(names):
            bounds.append(None)
            continue
        bounds.append(j)
        i = j
    out = []
    for k, (name, _) in enumerate(phases):
        if bounds[k] is None:
            continue
        nxt = next((b for b in bounds[k + 1:] if b is not None), None)
        s = int(ms[bounds[k]]["Start_Timestamp"])
        e = int(ms[nxt]["Start_Timestamp"]) if nxt is not None else t_end
        out.append((name, (e - s) / 1e6))
    # how much of the BLSTM recurrences' time other streams' kernels run
    # beside them (the recurrence holds 64 CUs; the rest are free for
    # weight gradients): overlapped ms / recurrence ms, forward and BPTT
    others = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                    for r in step if r["Queue_Id"] != main)
    rec = {}
    for kind, key in (("lstm_fwd_kernel", "fwd"), ("lstm_bwd_kernel", "bptt")):
        tot = ov = 0
        for r in ms:
            if kind not in r["Kernel_Name"]:
                continue
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            tot += b - a
            cov, cur = 0, a         # union of the other streams' intervals inside [a, b]
            for s0, e0 in others:
                s1, e1 = max(s0, cur), min(e0, b)
                if e1 > s1:
                    cov += e1 - s1
                    cur = e1
            ov += cov
        if tot:
            rec[key] = {"ms": round(tot / 1e6, 3), "overlapped_ms": round(ov / 1e6, 3),
                        "overlap_frac": round(ov / tot, 3)}
    return {"span_ms": (t_end - t0) / 1e6,
            "recurrence_overlap": rec,
            "busy_ms": {("main" if q == main else f"queue_{q}"): round(v, 3)
                        for q, v in busy.items()},
            "critical_path_ms": {n: round(v, 3) for n, v in out}}


def main():
    if sys.argv[1] == "--extract":
        step = load_step(sys.argv[2], which=int(sys.argv[4]) if len(sys.argv) > 4 else -2)
        with open(sys.argv[3], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(step[0].keys()))
            w.writeheader()
            w.writerows(step)
        return
    marker = sys.argv[2] if len(sys.argv) > 2 else "stft512_kernel"
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    step = load_step(sys.argv[1], marker, which)
    t0 = int(step[0]["Start_Timestamp"])
    t_end = max(int(r["End_Timestamp"]) for r in step)
    print(f"step span {(int(step[-1]['Start_Timestamp']) - t0) / 1e6:.3f} ms to last start, "
          f"{(t_end - t0) / 1e6:.3f} ms to last end, {len(step)} dispatches")
    queues = sorted({r["Queue_Id"] for r in step})
    for q in queues:
        ks = [r for r in step if r["Queue_Id"] == q]
        b = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks)
        print(f"queue {q}: {len(ks)} dispatches, busy {b / 1e6:.3f} ms")
    main_q = max(queues, key=lambda q: sum(1 for r in step if r["Queue_Id"] == q))
    print(f"\n(main queue = {main_q})  t_start(ms)  dur(ms)  gap_before(ms)  queue  kernel")
    prev_end = {}
    gap_total = 0
    for r in step:
        s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
        gap = (s - prev_end[q]) if q in prev_end else 0
        if q == main_q:
            gap_total += max(gap, 0)
        prev_end[q] = max(e, prev_end.get(q, 0))
        name = r["Kernel_Name"].replace("void ", "").replace("ainp::", "")[:70]
        print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} {gap / 1e6:8.3f}  {q:>3}  {name}")
    print(f"\nmain-queue idle gaps in the step: {gap_total / 1e6:.3f} ms")
    cp = critical_path(step)
    print("\ncritical path per phase (main stream):")
    for n, v in cp["critical_path_ms"].items():
        print(f"  {n:22s} {v:7.3f} ms")
    print(f"  {'sum':22s} {sum(cp['critical_path_ms'].values()):7.3f} ms  (span {cp['span_ms']:.3f})")
    print("recurrence overlap:", cp["recurrence_overlap"])


if __name__ == "__main__":
    main()
