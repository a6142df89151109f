#!/bin/bash
# A/B on one box: AINP_COUT1_STRIP (Cout=1 convs on the column-strip kernel), GAN C4 bf16 and C5.
set -o pipefail
OUT=gpurun_out/${1:-ab7}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gan.py -x -q --timeout 240 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
for v in 0 1; do
  AINP_COUT1_STRIP=$v timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline \
    --steps 30 > "$OUT/gan_strip_$v.$r.json" 2>&1 || exit 1
  echo "gan strip=$v: $(tail -1 $OUT/gan_strip_$v.$r.json | cut -c120-200)"
done
done
AINP_COUT1_STRIP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_bf16" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/gan_bf16.log" 2>&1 || exit 1
grep "ms/step" "$OUT/gan_bf16.log"
echo "all ok"
