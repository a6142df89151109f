#!/bin/bash
# rocprofv3 counter passes over the GAN bench's roofline kernel (the final
# PartialConv2d on conv_gen_x6_kernel, launched alone by
# tools/roofline_probe_gan.py): FETCH_SIZE and WRITE_SIZE in separate passes,
# then an SQ pass.  Also the per-layer conv_gen timer.  One pass per run.
#   gpurun -- bash tools/pmc_gan.sh <tag>
set -o pipefail
TAG=${1:-pmc_gan}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/roofline_probe_gan.py 5 > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES || exit 1
# algorithmic bytes: x0 8x64x192x320 + m0 8x192x320 + x1, m1, ratio 8x384x640 + out 8x64x384x640 (fp32)
ALG=$(( 4 * (8*64*192*320 + 8*192*320 + 3*8*384*640 + 8*64*384*640) ))
python3 tools/traffic_json.py "$OUT" conv_gen_x6 $ALG "tools/pmc_gan.sh over tools/roofline_probe_gan.py" \
  > "$OUT/traffic.json" && cat "$OUT/traffic.json"
python3 tools/pmc_table.py "$OUT"/sq/run_counter_collection.csv conv_gen_x6 > "$OUT/sq_table.txt"
cat "$OUT/sq_table.txt"
timeout -k 10 200 python3 tools/gan_layer_bench.py > "$OUT/layers.log" 2>&1 && tail -3 "$OUT/layers.log"
