#!/bin/bash
# SQ / traffic counter passes over the CNNBLSTM conv kernels alone
# (tools/conv_probe.py), one counter group per run.
#   gpurun -- bash tools/pmc_conv.sh <tag> [fp32|bf16] [pairs] [cl]
set -o pipefail
TAG=${1:-pmc_conv}
DT=${2:-fp32}
PAIRS=${3:-16-32,32-16,32-64,64-32}
LAY=${4:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/conv_probe.py 5 $DT $PAIRS $LAY > "$OUT/times.log" 2>&1 || exit 1
cat "$OUT/times.log"
pass() {
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/conv_probe.py 3 $DT $PAIRS $LAY > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
pass sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
python3 tools/pmc_table.py "$OUT"/sq/run_counter_collection.csv conv > "$OUT/sq_table.txt"
cat "$OUT/sq_table.txt"
