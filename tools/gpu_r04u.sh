#!/bin/bash
# Round 4: wide-conv split target 512 (default) vs 768 (AINP_CONV_SPLIT_WIDE=3), C4 / C5.
set -o pipefail
OUT=gpurun_out/${1:-r04u}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # tag clip env...
  local tag=$1 clip=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload gan --dtype bf16 --clip-s $clip \
    --no-cpu-baseline --steps 20 > "$OUT/$tag.json" 2> "$OUT/$tag.err" || return 1
  python - "$OUT/$tag.json" "$tag" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"),
              "wide", d.get("roofline_wide", {}).get("frac"), flush=True)
PY
}
for rep in 1 2 3; do
  run c4_t512_$rep 5 AINP_CONV_SPLIT_WIDE=1 || exit 1
  run c4_t768_$rep 5 AINP_CONV_SPLIT_WIDE=3 || exit 1
done
for rep in 1 2; do
  run c5_t512_$rep 8 AINP_CONV_SPLIT_WIDE=1 || exit 1
  run c5_t768_$rep 8 AINP_CONV_SPLIT_WIDE=3 || exit 1
done
AINP_CONV_SPLIT_WIDE=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gan.py > "$OUT/pytest_gan_768.log" 2>&1 || { tail -30 "$OUT/pytest_gan_768.log"; exit 1; }
tail -1 "$OUT/pytest_gan_768.log"
echo "all steps ok"
