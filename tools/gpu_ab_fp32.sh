#!/bin/bash
# C2 fp32 train step under environment variants, kernel-traced.
#   gpurun -- bash tools/gpu_ab_fp32.sh <tag> "VAR=a" "VAR=b" ...
set -o pipefail
OUT=gpurun_out/${1:-abf}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $i: $v"
  env $v timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/v$i" -o run -- \
    python3 tools/step_prof.py --steps 10 --dtype fp32 > "$OUT/v$i.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/v$i.log"
done
echo "all steps ok"
