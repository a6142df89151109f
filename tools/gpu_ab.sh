#!/bin/bash
# A/B pass: GAN ring conv tests + C4 bf16 benches ring/old, C2 benches pair-join on/off.
set -o pipefail
OUT=gpurun_out/${1:-ab}
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
step 500 pytest_gan.log python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_dconv16.py -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
step 200 gan_ring.json python bench.py --workload gan --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
AINP_CONV16_RING=0 step 200 gan_old.json python bench.py --workload gan --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
step 200 c2_nojoin.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
AINP_PAIR_JOIN=1 step 200 c2_join.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
step 200 c2_nojoin2.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-graph || exit 1
echo "all steps ok"
