#!/bin/bash
# bf16 layer-0 projection split 3 on the 256 tile: tests, bench A/B, kernel trace.
#   gpurun -- bash tools/gpu_b16split.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-b16s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "bf16nt or bf16" > "$OUT/t.log" 2>&1 || { tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
for v in 1 3 1 3 1 3; do
  AINP_B16_PROJ_SPLIT=$v timeout -k 10 200 python bench.py --dtype bf16 --no-cpu-baseline \
    > "$OUT/bench_s$v.$RANDOM.json" 2>/dev/null || exit 1
done
for v in 1 3; do
  AINP_B16_PROJ_SPLIT=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/ab$v" -o run -- \
    python3 tools/step_prof.py --steps 10 --dtype bf16 > "$OUT/ab$v.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/ab$v.log"
done
echo "all b16 steps ok"
