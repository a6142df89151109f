#!/bin/bash
# Round 6: the bf16 LDS-DMA 32 -> 64 weight gradient's variants (AINP_WDM_VARIANT:
# tile rows / ring stages) and measurement switches (AINP_WDM_DBG: 1 no MFMAs,
# 2 no prologue pass), each kernel-timed by rocprofv3 on tools/conv_probe.py.
#   gpurun -- bash tools/wdm_sweep.sh <tag> "<variants>" "<dbg modes>"
set -o pipefail
TAG=${1:?tag}; VARS=${2:-"0 1 2 3"}; DBGS=${3:-"0"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $VARS; do for d in $DBGS; do
  d_=$OUT/v${v}_d${d}
  AINP_WDM_VARIANT=$v AINP_WDM_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv \
    -d "$d_" -o run -- python3 tools/conv_probe.py 20 bf16 32-64 cl > "$d_.log" 2>&1 || { echo "v$v d$d failed"; exit 1; }
  f=$(find "$d_" -name "*kernel_stats.csv" | head -1)
  echo "variant $v dbg $d: $(grep -h wgrad_b16dma "$f" | awk -F'","' '{print $4}') ns avg"
done; done
