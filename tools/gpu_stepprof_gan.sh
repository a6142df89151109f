#!/bin/bash
# Per-step kernel tables of the GAN C4 step, fp32 and bf16.
set -o pipefail
OUT=gpurun_out/${1:-stepprof_gan}
mkdir -p "$OUT"
export TMPDIR=/tmp
for dt in bf16 fp32; do
  echo "== $dt"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$dt" -o run -- \
    python3 tools/step_prof.py --workload gan --steps 6 --dtype $dt > "$OUT/$dt.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/$dt.log"
done
echo "all steps ok"
