#!/bin/bash
# rocprofv3 counter passes over the GAN bench's roofline kernel (the final
# PartialConv2d, launched alone by tools/roofline_probe_gan.py): FETCH_SIZE and
# WRITE_SIZE in separate passes, then an SQ pass.  One pass per run.
#   gpurun -- bash tools/pmc_gan.sh <tag> [fp32|bf16]
set -o pipefail
TAG=${1:-pmc_gan}
DT=${2:-fp32}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/roofline_probe_gan.py 5 $DT > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES || exit 1
if [ "$DT" = bf16 ]; then
  # x0 bf16 NHWC 8x192x320x64 + expanded skip 8x384x640x32 bf16 + ratio fp32 8x384x640
  # + out fp32 8x64x384x640 + weights 64x608 bf16
  ALG=$(( 2 * 8*192*320*64 + 2 * 8*384*640*32 + 4 * 8*384*640 + 4 * 8*64*384*640 + 2 * 64*608 ))
  KN=conv_gen_nhwc16
else
  # x0 8x64x192x320 + m0 8x192x320 + x1, m1, ratio 8x384x640 + out 8x64x384x640 (fp32)
  ALG=$(( 4 * (8*64*192*320 + 8*192*320 + 3*8*384*640 + 8*64*384*640) ))
  KN=conv_gen_x6
fi
python3 tools/traffic_json.py "$OUT" $KN $ALG "tools/pmc_gan.sh $DT over tools/roofline_probe_gan.py" \
  > "$OUT/traffic.json" && cat "$OUT/traffic.json"
python3 tools/pmc_table.py "$OUT"/sq/run_counter_collection.csv $KN > "$OUT/sq_table.txt"
cat "$OUT/sq_table.txt"
