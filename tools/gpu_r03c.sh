#!/bin/bash
# conv16 variant 3 with BM=64 + CNNBLSTM bf16 per-step kernel table.
#   gpurun -- bash tools/gpu_r03c.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r03c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py -x -v --timeout 120 --timeout-method thread \
  -k "variants_bit_identical or nhwc16" > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/conv16_lab.py --variants 0,3,4 > "$OUT/lab_c4.log" 2>&1 || { tail -20 "$OUT/lab_c4.log"; exit 1; }
tail -2 "$OUT/lab_c4.log"
timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline > "$OUT/bench_gan_c4_bf16.json" 2>&1 || exit 1
tail -1 "$OUT/bench_gan_c4_bf16.json" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_bf16" -o run -- \
  python3 tools/step_prof.py --steps 10 --dtype bf16 > "$OUT/cnn_bf16.log" 2>&1 || exit 1
grep "ms/step" "$OUT/cnn_bf16.log"
for dt in fp32 bf16; do
  timeout -k 10 300 python3 tools/cnnblstm_op_bench.py $dt > "$OUT/opbench_$dt.log" 2>&1 || exit 1
  head -2 "$OUT/opbench_$dt.log" | tail -1
done
echo "all ok"
