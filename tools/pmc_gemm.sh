#!/bin/bash
# rocprofv3 counter passes over the bench's roofline kernel (the LSTM layer-0
# input projection GEMM, launched alone by tools/roofline_probe.py): HBM traffic
# (FETCH_SIZE, WRITE_SIZE in separate passes) and an SQ pass (clock, MFMA busy,
# wave-cycle split, LDS bank conflicts).  One pass per rocprofv3 run.
#   gpurun -- bash tools/pmc_gemm.sh <tag> [fp32|bf16]
set -o pipefail
TAG=${1:-pmc}
DT=${2:-fp32}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/roofline_probe.py 5 $DT > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES || exit 1
if [ "$DT" = bf16 ]; then
  # X [10688][16448] + W_cat [1024][16448] bf16 read once, three fp32 split-K
  # slabs [10688][1024] written (the slab sum is a separate launch)
  python3 tools/traffic_json.py "$OUT" gemm_bf16nt $(( 2 * (10688*16448 + 1024*16448) + 3 * 4 * 10688*1024 )) \
    "tools/pmc_gemm.sh bf16 over tools/roofline_probe.py" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
else
  # the 256x256 x6 tile, split 3: X [10688][16448] + W_ih (both) [1024][16448]
  # fp32 read once, three fp32 slabs [10688][1024] written (the slab sum is a
  # separate launch)
  python3 tools/traffic_json.py "$OUT" gemm_x6nt_256 $(( 4 * (10688*16448 + 1024*16448) + 3 * 4 * 10688*1024 )) \
    "tools/pmc_gemm.sh fp32 over tools/roofline_probe.py" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
fi
python3 tools/pmc_table.py "$OUT"/sq/run_counter_collection.csv gemm > "$OUT/sq_table.txt"
cat "$OUT/sq_table.txt"
