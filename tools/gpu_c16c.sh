#!/bin/bash
# conv16 variant 4 (64-deep K-tiles): bit-identity tests, per-layer lab, GAN bench.
set -o pipefail
OUT=gpurun_out/${1:-c16c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py -x -v --timeout 120 --timeout-method thread \
  -k "variants_bit_identical or nhwc16" > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/conv16_lab.py --variants 0,3,4 > "$OUT/lab_c4.log" 2>&1 || { tail -20 "$OUT/lab_c4.log"; exit 1; }
tail -3 "$OUT/lab_c4.log"
for v in 3 4; do
  AINP_CONV16=$v timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline --steps 30 \
    > "$OUT/bench_gan_v$v.json" 2>&1 || exit 1
  tail -1 "$OUT/bench_gan_v$v.json" | cut -c1-200
done
echo "all ok"
