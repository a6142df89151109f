#!/bin/bash
# A/B on one box: AINP_CONV_OUT16 (GAN bf16 C4), twice each.
set -o pipefail
OUT=gpurun_out/${1:-ab4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_kernels.py -x -q --timeout 240 \
  --timeout-method thread -k "nhwc16 or gan_step or epilogue" > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
for v in 0 1; do
  AINP_CONV_OUT16=$v timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline \
    --steps 30 > "$OUT/gan_out16_$v.$r.json" 2>&1 || exit 1
  echo "gan out16=$v: $(tail -1 $OUT/gan_out16_$v.$r.json | cut -c120-200)"
done
done
echo "all ok"
