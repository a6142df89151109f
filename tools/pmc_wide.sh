#!/bin/bash
# rocprofv3 counter passes over the GAN bf16 wide-tile conv on the bench's
# roofline_wide layer (U-Net decoder block 768 -> 256 at 48 x 80, B = 8: layer 10
# of tools/conv16_lab.py, launched 5 times alone after one recorded step):
# FETCH_SIZE and WRITE_SIZE in separate passes, then an SQ pass.
#   gpurun -- bash tools/pmc_wide.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-pmc_wide}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 180 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/conv16_lab.py --only 10 --variants 3 --reps 5 > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES || exit 1
# x0 8x24x40x512 + x1 8x48x80x256 bf16 NHWC, weights 256x6912 bf16, ratio 8x48x80 fp32,
# out 8x256x48x80 fp32, BN partials 240x2x256 fp64
ALG=$(( 2*8*24*40*512 + 2*8*48*80*256 + 2*256*6912 + 4*8*48*80 + 4*8*256*48*80 + 8*240*2*256 ))
KN="conv_gen_nhwc16_wide_kernel<256"
python3 tools/traffic_json.py "$OUT" "$KN" $ALG "tools/pmc_wide.sh over tools/conv16_lab.py --only 10" 4 \
  > "$OUT/traffic.json" && cat "$OUT/traffic.json"
python3 tools/pmc_table.py "$OUT"/sq/run_counter_collection.csv "$KN" 5 > "$OUT/sq_table.txt"
cat "$OUT/sq_table.txt"
echo "all ok"
