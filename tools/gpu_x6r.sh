#!/bin/bash
# x6r (csrc/gemm_x6r.hip) check + A/B: new GEMM tests, the kernel probe, then
# C2 benches with the fused layer-0 backward pair on/off.
set -o pipefail
OUT=gpurun_out/${1:-x6r}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -4 "$OUT/$log" | cut -c1-300
  return $rc
}
step 400 pytest_x6r.log python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 240 --timeout-method thread -k "x6" || exit 1
step 200 probe.log python tools/x6r_probe.py 10 || exit 1
step 200 bench_new.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
AINP_L0_BWD_X6R=0 step 200 bench_old.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
AINP_X6R_FWD=1 step 200 bench_fwd.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
echo "all steps ok"
