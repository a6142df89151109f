#!/bin/bash
# Round 4: U-Net BatchNorm pass without the fp32 write-back (AINP_AFFINE_NO_Y):
# parity, C4 / C5 A/B, step table.
set -o pipefail
OUT=gpurun_out/${1:-r04z6}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gan.py > "$OUT/pytest_gan.log" 2>&1 || { tail -30 "$OUT/pytest_gan.log"; exit 1; }
tail -2 "$OUT/pytest_gan.log"
run() {  # tag clip env...
  local tag=$1 clip=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload gan --dtype bf16 --clip-s $clip \
    --no-cpu-baseline --steps 20 > "$OUT/$tag.json" 2> "$OUT/$tag.err" || return 1
  python - "$OUT/$tag.json" "$tag" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["ms_per_step"], "ms/step median", d.get("ms_per_step_median"), flush=True)
PY
}
for rep in 1 2 3; do
  run c4_noy1_$rep 5 AINP_AFFINE_NO_Y=1 || exit 1
  run c4_noy0_$rep 5 AINP_AFFINE_NO_Y=0 || exit 1
done
for rep in 1 2; do
  run c5_noy1_$rep 8 AINP_AFFINE_NO_Y=1 || exit 1
  run c5_noy0_$rep 8 AINP_AFFINE_NO_Y=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/step" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/step.log" 2>&1 || exit 1
echo "all steps ok"
