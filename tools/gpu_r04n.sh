#!/bin/bash
# Round 4: channel-last bf16 copies written by the few-input-channel conv and
# by the VGG max-pool (AINP_OUT16_DIRECT): tests, C4 A/B, kernel summary.
set -o pipefail
OUT=gpurun_out/${1:-r04n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gan.py tests/test_gpu_dconv16.py > "$OUT/pytest_gan.log" 2>&1 || { tail -30 "$OUT/pytest_gan.log"; exit 1; }
tail -3 "$OUT/pytest_gan.log"
for rep in 1 2 3; do
  for d in 0 1; do
    AINP_OUT16_DIRECT=$d timeout -k 10 300 python bench.py --workload gan --dtype bf16 \
      --no-cpu-baseline --steps 20 > "$OUT/c4_d${d}_$rep.json" 2> "$OUT/c4_d${d}_$rep.err" || exit 1
    python - "$OUT/c4_d${d}_$rep.json" "direct$d rep$rep" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python bench.py --workload gan --dtype bf16 --no-cpu-baseline --steps 10 > "$OUT/prof.log" 2>&1 || exit 1
timeout -k 10 300 python tools/glue_sites.py > "$OUT/glue_sites.log" 2>&1 || { tail -20 "$OUT/glue_sites.log"; exit 1; }
grep -v amdgpu.ids "$OUT/glue_sites.log"
echo "all steps ok"
