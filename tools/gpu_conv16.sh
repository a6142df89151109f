#!/bin/bash
# conv_gen_nhwc16 variants: bit-identity tests, per-layer lab (C4 and C5), GAN
# bf16 bench per variant.   gpurun -- bash tools/gpu_conv16.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-conv16}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py -x -v --timeout 120 --timeout-method thread \
  -k "variants_bit_identical or nhwc16" > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/conv16_lab.py --variants 0,2,3 > "$OUT/lab_c4.log" 2>&1 || { tail -20 "$OUT/lab_c4.log"; exit 1; }
tail -4 "$OUT/lab_c4.log"
for v in 0 3; do
  AINP_CONV16=$v timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline --steps 30 \
    > "$OUT/bench_gan_v$v.json" 2>&1 || exit 1
  tail -1 "$OUT/bench_gan_v$v.json" | cut -c1-200
done
echo "all ok"
