#!/bin/bash
# GAN bf16 chain changes: GAN GPU tests, C4 / C5 bf16 benches, bf16 step kernel table.
set -o pipefail
OUT=gpurun_out/${1:-gan16}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_dconv16.py -x -v --timeout 240 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline > "$OUT/bench_gan_c4_bf16.json" 2>&1 || exit 1
tail -1 "$OUT/bench_gan_c4_bf16.json" | cut -c1-220
timeout -k 10 300 python bench.py --workload gan --clip-s 8 --dtype bf16 --no-cpu-baseline > "$OUT/bench_gan_c5.json" 2>&1 || exit 1
tail -1 "$OUT/bench_gan_c5.json" | cut -c1-220
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/bf16" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/bf16.log" 2>&1 || exit 1
grep "ms/step" "$OUT/bf16.log"
echo "all ok"
