#!/bin/bash
# Round 4: LDS-tiled Cout=1 conv (AINP_COUT1_TILED) for the generator's last
# PartialConv2d: parity tests, C4 A/B, per-step kernel table.
set -o pipefail
OUT=gpurun_out/${1:-r04r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gan.py > "$OUT/pytest_gan.log" 2>&1 || { tail -30 "$OUT/pytest_gan.log"; exit 1; }
tail -3 "$OUT/pytest_gan.log"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload gan --dtype bf16 \
    --no-cpu-baseline --steps 20 > "$OUT/c4_$tag.json" 2> "$OUT/c4_$tag.err" || return 1
  python - "$OUT/c4_$tag.json" "$tag" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
}
for rep in 1 2 3; do
  run tiled1_$rep AINP_COUT1_TILED=1 || exit 1
  run tiled0_$rep AINP_COUT1_TILED=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/step" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/step.log" 2>&1 || exit 1
grep "ms/step" "$OUT/step.log"
echo "all steps ok"
