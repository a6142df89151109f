#!/bin/bash
# Round 4: fused BatchNorm reduce + finalize, cached dgrad16 weights, Adam version bumps:
# parity, C2 / C4 / C5 benches, per-step kernel table.
set -o pipefail
OUT=gpurun_out/${1:-r04x}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gan.py tests/test_gpu_dconv16.py > "$OUT/pytest_gan.log" 2>&1 || { tail -30 "$OUT/pytest_gan.log"; exit 1; }
tail -2 "$OUT/pytest_gan.log"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "sum_slabs or splitk or bf16nt or reduce_finalize or adam or bn_" > "$OUT/pytest_k.log" 2>&1 || { tail -30 "$OUT/pytest_k.log"; exit 1; }
tail -2 "$OUT/pytest_k.log"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py > "$OUT/pytest_model.log" 2>&1 || { tail -30 "$OUT/pytest_model.log"; exit 1; }
tail -2 "$OUT/pytest_model.log"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > "$OUT/c2_$rep.json" 2> "$OUT/c2_$rep.err" || exit 1
  grep -o '"ms_per_step": [0-9.]*' "$OUT/c2_$rep.json"
done
for rep in 1 2 3; do
  for clip in 5 8; do
    timeout -k 10 300 python bench.py --workload gan --dtype bf16 --clip-s $clip --no-cpu-baseline \
      --steps 20 > "$OUT/gan_${clip}_$rep.json" 2> "$OUT/gan_${clip}_$rep.err" || exit 1
    python - "$OUT/gan_${clip}_$rep.json" "clip$clip rep$rep" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/step" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/step.log" 2>&1 || exit 1
grep "ms/step" "$OUT/step.log"
echo "all steps ok"
