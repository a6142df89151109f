#!/bin/bash
# Round 4: STFT feature kernel at three workgroups per CU (AINP_STFT_OCC=3):
# parity with it on, roofline_stft A/B.
set -o pipefail
OUT=gpurun_out/${1:-r04s}
mkdir -p "$OUT"
export TMPDIR=/tmp
AINP_STFT_OCC=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests -k "stft or feature" > "$OUT/pytest_stft_occ3.log" 2>&1 || { tail -30 "$OUT/pytest_stft_occ3.log"; exit 1; }
tail -2 "$OUT/pytest_stft_occ3.log"
for rep in 1 2 3; do
  for o in 2 3; do
    AINP_STFT_OCC=$o timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      --roofline-reps 50 > "$OUT/c2_occ${o}_$rep.json" 2> "$OUT/c2_occ${o}_$rep.err" || exit 1
    python - "$OUT/c2_occ${o}_$rep.json" "occ$o rep$rep" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        r = d["roofline_stft"]
        print(sys.argv[2], "stft", r["avg_launch_ms"], "ms frac", r["frac"], "step", d["ms_per_step"], flush=True)
PY
  done
done
echo "all steps ok"
