#!/bin/bash
# A/B pass: output-projection backward on x6r (tests + C2 benches: deferred
# weight gradient / joint launch / gemm_f32).
set -o pipefail
OUT=gpurun_out/${1:-ab2}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -2 "$OUT/$log" | cut -c1-300
  return $rc
}
step 600 pytest.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_dist.py -m gpu -x -v --timeout 240 --timeout-method thread -k "proj or x6 or cnnblstm or curve or model or step" || exit 1
step 200 c2_defer.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
AINP_PROJ_JOINT=1 step 200 c2_joint.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
AINP_PROJ_X6R=0 step 200 c2_f32.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
step 200 c2_defer2.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
echo "all steps ok"
