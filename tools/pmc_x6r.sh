#!/bin/bash
# rocprofv3 counter passes over the x6r GEMM (csrc/gemm_x6r.hip): the layer-0
# projection (the bench's roofline kernel) and the fused backward pair, each
# launched alone by tools/roofline_probe.py.  HBM traffic (FETCH_SIZE,
# WRITE_SIZE in separate passes) and an SQ pass.  One pass per rocprofv3 run.
#   gpurun -- bash tools/pmc_x6r.sh <tag>
set -o pipefail
TAG=${1:-pmc_x6r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <probe-mode> <counters...>
  local nm=$1 mode=$2; shift 2
  echo "== $(date +%T) pmc $nm ($mode): $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/roofline_probe.py 5 $mode > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
SQ="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
for mode in ${MODES:-fp32 pair}; do
  mkdir -p "$OUT/$mode"
  pass $mode/fetch $mode FETCH_SIZE || exit 1
  pass $mode/write $mode WRITE_SIZE || exit 1
  pass $mode/sq $mode $SQ || exit 1
  python3 tools/pmc_table.py "$OUT/$mode/sq/run_counter_collection.csv" gemm_x6r > "$OUT/$mode/sq_table.txt"
  cat "$OUT/$mode/sq_table.txt"
done
# algorithmic bytes per launch: projection = X [10688][16448] + W_ih (both)
# [1024][16448] fp32 read once + three fp32 slabs [10688][1024] written;
# pair = dg [10688][1024] + X + W_ih read once, dX [10688][16448] + dW_ih
# [1024][16448] written
if [ -n "$MODES" ]; then
  for mode in $MODES; do python3 tools/traffic_json.py "$OUT/$mode" gemm_x6r $(( 4 * (10688*1024 + 10688*16448 + 1024*16448) )) "tools/pmc_x6r.sh over tools/roofline_probe.py 5 $mode" > "$OUT/traffic_$mode.json"; done
  echo "all steps ok"; exit 0
fi
python3 tools/traffic_json.py "$OUT/fp32" gemm_x6r $(( 4 * (10688*16448 + 1024*16448) + 3 * 4 * 10688*1024 )) \
  "tools/pmc_x6r.sh over tools/roofline_probe.py 5 fp32" > "$OUT/traffic_fwd.json" && cat "$OUT/traffic_fwd.json" || exit 1
python3 tools/traffic_json.py "$OUT/pair" gemm_x6r $(( 4 * (10688*1024 + 2 * 10688*16448 + 2 * 1024*16448) )) \
  "tools/pmc_x6r.sh over tools/roofline_probe.py 5 pair" > "$OUT/traffic_pair.json" && cat "$OUT/traffic_pair.json"
echo "all steps ok"
