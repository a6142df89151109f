#!/bin/bash
# Round 4: Cout <= 64 bf16 convs on the LDS-DMA ring kernel (AINP_CONV16_SMALLCO=1) vs the register-staged kernel, C4 / C5.
set -o pipefail
OUT=gpurun_out/${1:-r04v1}
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
  run c4_sc0_$rep 5 AINP_CONV16_SMALLCO=0 || exit 1
  run c4_sc1_$rep 5 AINP_CONV16_SMALLCO=1 || exit 1
done
for rep in 1 2; do
  run c5_sc0_$rep 8 AINP_CONV16_SMALLCO=0 || exit 1
  run c5_sc1_$rep 8 AINP_CONV16_SMALLCO=1 || exit 1
done
AINP_CONV16_SMALLCO=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gan.py > "$OUT/pytest_gan_sc1.log" 2>&1 || { tail -30 "$OUT/pytest_gan_sc2.log"; exit 1; }
tail -1 "$OUT/pytest_gan_sc1.log"
echo "all steps ok"
