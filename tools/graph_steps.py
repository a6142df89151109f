"""Per-step summary of a rocprofv3 --kernel-trace CSV of `bench.py` (eager
steps, then the HIP-graph replays of the same step): span, dispatches,
hardware queues and each queue's busy time, the union of busy time (how much
the queues overlap) and whether the step ran the capturable Adam (graph).
Round 6 (why the replay is slower than eager).

  python tools/graph_steps.py run_kernel_trace.csv [marker]"""
import csv
import sys


def union_ms(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot / 1e6


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "stft512_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    for k, a in enumerate(idx):
        b = idx[k + 1] if k + 1 < len(idx) else len(rows)
        st = rows[a:b]
        if not any("adam_kernel" in r["Kernel_Name"] for r in st):
            continue   # evaluation passes (no optimizer)
        t0 = int(st[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in st)
        qs = sorted({r["Queue_Id"] for r in st})
        busy = {q: round(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                             for r in st if r["Queue_Id"] == q) / 1e6, 3) for q in qs}
        cnt = {q: sum(1 for r in st if r["Queue_Id"] == q) for q in qs}
        tot = sum(busy.values())
        un = union_ms([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in st])
        graph = any("adam_prologue" in r["Kernel_Name"] for r in st)
        print(f"step {k:2d} {'graph' if graph else 'eager'} span {(t1 - t0) / 1e6:7.3f} ms  "
              f"kernels {len(st):4d}  busy sum {tot:7.3f}  union {un:7.3f}  "
              f"overlap {tot - un:6.3f}  queues {dict((q, (busy[q], cnt[q])) for q in qs)}")


if __name__ == "__main__":
    main()
