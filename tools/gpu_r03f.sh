#!/bin/bash
# Round-3 final pass: full GPU suite, smoke, C2 / C3-shape / C4 / C5 benches,
# rocprofv3 kernel stats of the C2 bench, GAN bf16 and CNNBLSTM bf16 step tables.
#   gpurun -- bash tools/gpu_r03f.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r03f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -1 "$OUT/$log" | cut -c1-250
  return $rc
}
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step 300 bench.json python bench.py || exit 1
step 300 bench_bf16.json python bench.py --dtype bf16 --no-cpu-baseline || exit 1
step 300 bench_gan_c4_bf16.json python bench.py --workload gan --dtype bf16 --no-cpu-baseline || exit 1
step 300 bench_gan_c5.json python bench.py --workload gan --clip-s 8 --dtype bf16 --no-cpu-baseline || exit 1
step 300 prof.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-graph || exit 1
step 300 gan_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_bf16" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 || exit 1
step 300 cnn_bf16.log rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_bf16" -o run -- \
  python3 tools/step_prof.py --steps 10 --dtype bf16 || exit 1
echo "all steps ok"
