#!/bin/bash
# A/B: AINP_X6_HIOCC (bf16 C3 shape) and AINP_BENCH_CAPTURABLE (C2), one box.
set -o pipefail
OUT=gpurun_out/${1:-ab3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "conv3x3_bf16" > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
AINP_X6_HIOCC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 \
  --timeout-method thread -k "conv3x3_bf16" > "$OUT/pytest_hi.log" 2>&1 || { tail -5 "$OUT/pytest_hi.log"; exit 1; }
tail -1 "$OUT/pytest_hi.log"
for r in 1 2; do
for v in 0 1; do
  AINP_X6_HIOCC=$v timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline --no-graph --steps 30 \
    > "$OUT/bf16_hi$v.$r.json" 2>&1 || exit 1
  echo "bf16 hi=$v: $(tail -1 $OUT/bf16_hi$v.$r.json | cut -c100-200)"
  AINP_BENCH_CAPTURABLE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 \
    > "$OUT/c2_cap$v.$r.json" 2>&1 || exit 1
  echo "c2 cap=$v: $(tail -1 $OUT/c2_cap$v.$r.json | cut -c100-200)"
done
done
echo "all ok"
