#!/bin/bash
# GAN bf16 step profile + SQ counters of conv_gen_nhwc16 layers under variant 3.
#   gpurun -- bash tools/gpu_ganprof.sh <tag> [layer...]
set -o pipefail
OUT=gpurun_out/${1:-ganprof}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bf16" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/bf16.log" 2>&1 || exit 1
grep "ms/step" "$OUT/bf16.log"
for L in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -f csv \
    -d "$OUT/sq_l$L" -o run -- python3 tools/conv16_lab.py --only $L --variants 3 --reps 5 \
    > "$OUT/sq_l$L.log" 2>&1 || exit 1
  tail -1 "$OUT/sq_l$L.log"
done
echo "all ok"
