#!/bin/bash
# Round-2 closing pass: bf16 step A/B of the 256x256 GEMM, then the C2 bench,
# a rocprofv3 kernel trace of it, and the GAN fp32 (C4) and bf16 C5 benches.
#   gpurun -- bash tools/gpu_final.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -1 "$OUT/$log" | cut -c1-300
  return $rc
}
for v in 1 0; do
  step 240 ab$v.log env AINP_GEMM16_256=$v rocprofv3 --kernel-trace --stats -f csv -d "$OUT/ab$v" -o run -- \
    python3 tools/step_prof.py --steps 10 --dtype bf16 || exit 1
done
step 300 bench.json python bench.py || exit 1
step 300 prof.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit 1
step 300 bench_gan_fp32.json python bench.py --workload gan --no-cpu-baseline || exit 1
step 300 bench_gan_c5.json python bench.py --workload gan --dtype bf16 --clip-s 8 --no-cpu-baseline || exit 1
echo "all steps ok"
