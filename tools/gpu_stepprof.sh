#!/bin/bash
# Per-step kernel tables of the C2 (fp32) and C3-shape (bf16) train steps.
#   gpurun -- bash tools/gpu_stepprof.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-stepprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
for dt in fp32 bf16; do
  echo "== $dt"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$dt" -o run -- \
    python3 tools/step_prof.py --steps 10 --dtype $dt > "$OUT/$dt.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/$dt.log"
done
echo "all steps ok"
