#!/bin/bash
# A/B on one box: AINP_X6R_EARLY (tile kt+2's DMA right after the barrier) --
# x6r parity tests, the layer-0 GEMMs alone (x6r_probe) and the C2 bench, twice.
set -o pipefail
OUT=gpurun_out/${1:-ab6}
mkdir -p "$OUT"
export TMPDIR=/tmp
AINP_X6R_EARLY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 240 \
  --timeout-method thread -k "x6r or l0_bwd_x6 or proj_bwd_x6 or x6_multi" > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
for v in 0 1; do
  AINP_X6R_EARLY=$v timeout -k 10 200 python tools/x6r_probe.py 10 > "$OUT/probe_$v.$r.log" 2>&1 || exit 1
  echo "probe early=$v: $(grep -E 'fwd_x6r|pair_x6r' $OUT/probe_$v.$r.log | tr '\n' ' ')"
  AINP_X6R_EARLY=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 \
    > "$OUT/c2_early_$v.$r.json" 2>&1 || exit 1
  echo "c2 early=$v: $(tail -1 $OUT/c2_early_$v.$r.json | cut -c100-200)"
done
done
echo "all ok"
