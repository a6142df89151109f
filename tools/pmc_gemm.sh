#!/bin/bash
# rocprofv3 counter passes over the bench's roofline kernel (the LSTM layer-0
# input projection GEMM, launched alone by tools/roofline_probe.py): HBM traffic
# (FETCH_SIZE, WRITE_SIZE in separate passes) and an SQ pass (clock, MFMA busy,
# wave-cycle split, LDS bank conflicts).  One pass per rocprofv3 run.
#   gpurun -- bash tools/pmc_gemm.sh <tag>
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/roofline_probe.py 5 > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES || exit 1
python3 tools/traffic_json.py "$OUT" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
python3 tools/pmc_table.py "$OUT"/sq/run_counter_collection.csv gemm > "$OUT/sq_table.txt"
cat "$OUT/sq_table.txt"
