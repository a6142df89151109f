#!/bin/bash
# layer-0 fp32 dX on the 256 tile: GPU suite, bench A/B and kernel trace.
#   gpurun -- bash tools/gpu_dx.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-dx}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for v in 0 1 0 1; do
  AINP_DX_X6_256=$v timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/bench_dx$v.$RANDOM.json" 2>/dev/null || exit 1
done
bash tools/gpu_ab_fp32.sh ${1:-dx}/ab "AINP_DX_X6_256=0" "AINP_DX_X6_256=1" || exit 1
echo "all dx steps ok"
