#!/bin/bash
# Round 4: STFT one-tile-ahead clean-frame loads (parity + roofline_stft), and
# the x6p/x6q two-step halo prefetch A/B (AINP_X6_PF=1|2) on the conv probe and
# the C2 / C3-shape benches.
set -o pipefail
OUT=gpurun_out/${1:-r04g}
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
step 300 pytest_stft.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_istft.py -v --timeout 120 --timeout-method thread -k "stft or gap_frames or gl_" || exit 1
for pf in 1 2; do
  for dt in fp32 bf16; do
    AINP_X6_PF=$pf step 120 probe_${dt}_pf$pf.log python tools/conv_probe.py 5 $dt 16-32,32-16,32-64 || exit 1
    grep -v amdgpu.ids "$OUT/probe_${dt}_pf$pf.log"
  done
done
AINP_X6_PF=2 step 600 pytest_conv_pf2.log python -u -m pytest tests/test_gpu_kernels.py -v --timeout 120 --timeout-method thread -k "conv" || exit 1
for pf in 1 2 1 2; do
  AINP_X6_PF=$pf step 300 bench_fp32_pf$pf.json python bench.py --no-cpu-baseline --steps 30 || exit 1
  AINP_X6_PF=$pf step 300 bench_bf16_pf$pf.json python bench.py --dtype bf16 --no-cpu-baseline --no-graph --steps 30 || exit 1
done
echo "all steps ok"
