#!/bin/bash
# GAN bf16 step under conv_gen variants (env settings passed as arguments).
#   gpurun -- bash tools/gpu_ganvar.sh <tag> "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
OUT=gpurun_out/${1:-ganvar}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $i: $v"
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/v$i" -o run -- \
    python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/v$i.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/v$i.log"
done
echo "all steps ok"
