#!/bin/bash
# Round 4: row-staged im2col16 (AINP_IM2COL16_ROWS) for the GAN discriminator
# backward: bit-exactness tests, C4 A/B and a kernel summary of each.
set -o pipefail
OUT=gpurun_out/${1:-r04m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_dconv16.py > "$OUT/pytest_dconv16.log" 2>&1 || { tail -30 "$OUT/pytest_dconv16.log"; exit 1; }
tail -3 "$OUT/pytest_dconv16.log"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "ntcf or bn_relu" > "$OUT/pytest_ntcf.log" 2>&1 || { tail -30 "$OUT/pytest_ntcf.log"; exit 1; }
tail -3 "$OUT/pytest_ntcf.log"
for rep in 1 2 3; do
  for rows in 0 1; do
    AINP_IM2COL16_ROWS=$rows timeout -k 10 300 python bench.py --workload gan --dtype bf16 \
      --no-cpu-baseline --steps 20 > "$OUT/c4_rows${rows}_$rep.json" 2> "$OUT/c4_rows${rows}_$rep.err" || exit 1
    python - "$OUT/c4_rows${rows}_$rep.json" "rows$rows rep$rep" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
  done
done
for rows in 0 1; do
  AINP_IM2COL16_ROWS=$rows timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rows$rows" \
    -o run -- python bench.py --workload gan --dtype bf16 --no-cpu-baseline --steps 10 \
    > "$OUT/prof_rows$rows.log" 2>&1 || exit 1
done
find "$OUT" -name '*kernel_stats.csv' | while read f; do
  echo "== $f"; grep -i "im2col\|gemm_bf16" "$f" | cut -d, -f1-5
done
timeout -k 10 300 python tools/glue_sites.py > "$OUT/glue_sites.log" 2>&1 || { tail -20 "$OUT/glue_sites.log"; exit 1; }
grep -v amdgpu.ids "$OUT/glue_sites.log"
echo "all steps ok"
