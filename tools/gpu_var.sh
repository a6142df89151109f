#!/bin/bash
# tools/step_prof.py under env-selected kernel variants, each in its own
# rocprofv3 kernel-trace run.
#   gpurun -- bash tools/gpu_var.sh <tag> "<step_prof args>" "VAR=a" "VAR=b VAR2=c" ...
set -o pipefail
OUT=gpurun_out/${1:-var}; shift
ARGS=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $i: $v :: $ARGS"
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/v$i" -o run -- \
    python3 tools/step_prof.py $ARGS > "$OUT/v$i.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/v$i.log"
done
echo "all steps ok"
