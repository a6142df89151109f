#!/bin/bash
# rocprofv3 HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: one pass each) over
# the fused STFT/feature/mask kernel launched alone (tools/stft_probe.py).
#   gpurun -- bash tools/pmc_stft.sh <tag>
set -o pipefail
TAG=${1:-pmc_stft}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local nm=$1; shift
  echo "== $(date +%T) pmc $nm: $*"
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d "$OUT/$nm" -o run -- \
    python3 tools/stft_probe.py 6 > "$OUT/$nm.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
if [ "${2:-}" = sq ]; then
  pass sq GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU || exit 1
  exit 0
fi
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
python3 tools/traffic_json.py "$OUT" stft512 52157440 "tools/pmc_stft.sh over tools/stft_probe.py" \
  > "$OUT/traffic.json" && cat "$OUT/traffic.json"
