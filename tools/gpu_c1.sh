#!/bin/bash
# LDS-tiled Cout=1 conv: parity tests, A/B against the per-pixel kernel, the
# (AINP_COUT1_TILE selected the LDS-tiled Cout=1 kernel of that A/B; the kernel was dropped.)
# GAN C4 step with both, then the 2-rank gloo DP rehearsal (tools/gpu_dp2.sh).
set -o pipefail
OUT=gpurun_out/${1:-c1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gan.log" 2>&1 || { tail -30 "$OUT/pytest_gan.log"; exit 1; }
tail -1 "$OUT/pytest_gan.log"
AINP_COUT1_TILE=0 timeout -k 10 120 python -u tools/cout1_ab.py pixel > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
timeout -k 10 120 python -u tools/cout1_ab.py tile >> "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
for v in 0 1 0 1; do
  AINP_COUT1_TILE=$v timeout -k 10 300 python bench.py --workload gan --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/c4_tile$v.json" 2> "$OUT/c4_tile$v.err" || { tail -5 "$OUT/c4_tile$v.err"; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/c4_tile$v.json').read().strip().splitlines()[-1]);print('tile=$v',d['ms_per_step'])"
done
bash tools/gpu_dp2.sh ${1:-c1}/dp2
