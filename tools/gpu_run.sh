#!/bin/bash
# Generic GPU-box runner: each argument is "<seconds>:<log>:<command>"; every
# step runs under its own time limit and the chain stops at the first failure.
#   gpurun --timeout 900 -- bash tools/gpu_run.sh <tag> "600:pytest.log:python -m pytest ..." ...
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  t=${spec%%:*}; rest=${spec#*:}; log=${rest%%:*}; cmd=${rest#*:}
  echo "== $(date +%T) $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$log" 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
echo "all steps ok"
