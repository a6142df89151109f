#!/bin/bash
# Same-box comparison of bench.py under several environment settings, run
# round-robin <reps> times.
#   gpurun -- bash tools/gpu_ab_multi.sh <tag> <reps> "<bench args>" "name=ENV1,ENV2" ...
# e.g.  bash tools/gpu_ab_multi.sh r05i 2 "--dtype bf16" "base=" "free8=AINP_SIDE_FREE_CUS=8"
set -o pipefail
OUT=gpurun_out/${1:?tag}
REPS=${2:-2}
BARGS=${3:-}
shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name envlist rep
  local name=$1 envs=${2//,/ } rep=$3
  env $envs timeout -k 10 300 python bench.py $BARGS --no-cpu-baseline --steps 20 \
    > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { tail -20 "$OUT/${name}_$rep.err"; return 1; }
  python - "$OUT/${name}_$rep.json" "$name" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
}
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    run "${v%%=*}" "${v#*=}" $rep || exit 1
  done
done
echo "all steps ok"
