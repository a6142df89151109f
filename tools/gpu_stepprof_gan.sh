#!/bin/bash
# Per-step kernel tables of the GAN bf16 steps the bench times: C4 (5 s clips,
# T=626) and C5 (8 s clips, T=1001); 3 warm-up + 10 timed steps, so the
# tables divide by 13 (bench.py STEP_TABLES).
#   gpurun -- bash tools/gpu_stepprof_gan.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-stepprof_gan}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in "c4 5" "c5 8"; do
  set -- $c
  echo "== $1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$1" -o run -- \
    python3 tools/step_prof.py --workload gan --steps 10 --dtype bf16 --clip-s $2 > "$OUT/$1.log" 2>&1 || exit 1
  grep "ms/step" "$OUT/$1.log"
done
echo "all steps ok"
