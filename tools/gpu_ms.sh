#!/bin/bash
# GAN step A/B on one box (AINP_SN_FOREACH; first used for AINP_MASK_SIDE,
# profiles/r03_ms_summary.txt, dropped): GAN GPU tests, C4 and C5 bf16 benches.
set -o pipefail
OUT=gpurun_out/${1:-ms}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_dist.py -x -v --timeout 200 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in 0 1 0 1; do
  AINP_SN_FOREACH=$v timeout -k 10 300 python bench.py --workload gan --dtype bf16 --steps 20 --warmup 5 \
    --no-cpu-baseline > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || { tail -5 "$OUT/c4_$v.err"; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c4_$v.json').read().strip().splitlines()[-1]);print('C4 sn_foreach=$v',d['ms_per_step'],d['ms_per_step_median'])"
done
for v in 0 1; do
  AINP_SN_FOREACH=$v timeout -k 10 300 python bench.py --workload gan --clip-s 8 --dtype bf16 --steps 20 \
    --warmup 5 --no-cpu-baseline > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err" || { tail -5 "$OUT/c5_$v.err"; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c5_$v.json').read().strip().splitlines()[-1]);print('C5 sn_foreach=$v',d['ms_per_step'],d['ms_per_step_median'])"
done
echo "all ok"
