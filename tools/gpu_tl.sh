#!/bin/bash
# Kernel trace of the C2 step (step_prof.py) for per-stream timelines.
#   gpurun -- bash tools/gpu_tl.sh <tag> [fp32|bf16]
set -o pipefail
OUT=gpurun_out/${1:-tl}
DT=${2:-fp32}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$DT" -o run -- \
  python3 tools/step_prof.py --steps 6 --dtype $DT > "$OUT/$DT.log" 2>&1 || exit 1
grep "ms/step" "$OUT/$DT.log"
TR=$(ls "$OUT/$DT"/*/run_kernel_trace.csv 2>/dev/null | head -1)
[ -z "$TR" ] && TR=$(ls "$OUT/$DT"/run_kernel_trace.csv)
python3 tools/stream_timeline.py "$TR" > "$OUT/${DT}_timeline.txt"
echo "all steps ok"
