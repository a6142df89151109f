#!/bin/bash
# Generic same-box A/B of bench.py under two environment settings, alternating.
#   gpurun -- bash tools/gpu_ab_env.sh <tag> <reps> "<bench args>" "<env A>" "<env B>" [pytest args]
# e.g.  bash tools/gpu_ab_env.sh r05d 3 "--dtype bf16" "AINP_Y16=0" "AINP_Y16=1"
# Optional 6th argument: a pytest selection run first (under env B), e.g.
#   "tests/test_gpu_model.py -k bf16".
set -o pipefail
OUT=gpurun_out/${1:?tag}
REPS=${2:-2}
BARGS=${3:-}
ENVA=${4:-}
ENVB=${5:-}
PYT=${6:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$PYT" ]; then
  env $ENVB timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    -m gpu $PYT > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
run() {  # tag env
  local tag=$1; shift
  env $@ timeout -k 10 300 python bench.py $BARGS --no-cpu-baseline --steps 20 \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || return 1
  python - "$OUT/$tag.json" "$tag" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
}
for rep in $(seq 1 $REPS); do
  run A_$rep $ENVA || exit 1
  run B_$rep $ENVB || exit 1
done
echo "all steps ok"
