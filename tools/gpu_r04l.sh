#!/bin/bash
# Round 4: order of the deferred decoder / output-projection weight gradients
# (AINP_DEFER_LIFO) and the projection's joint backward (AINP_PROJ_JOINT) vs
# the layer-0 backward pair's in-step contention: C2 / C3-shape benches.
set -o pipefail
OUT=gpurun_out/${1:-r04l}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # cfg tag env...
  local cfg=$1 tag=$2; shift 2
  local extra=""
  [ "$cfg" = c3 ] && extra="--dtype bf16"
  env "$@" timeout -k 10 300 python bench.py $extra --no-cpu-baseline --no-graph --steps 30 > "$OUT/${cfg}_$tag.json" 2> "$OUT/${cfg}_$tag.err" || return 1
  python - "$OUT" "$cfg" "$tag" <<'PY'
import json, sys
out, cfg, tag = sys.argv[1:]
for l in open(f"{out}/{cfg}_{tag}.json"):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{cfg} {tag}: {d['ms_per_step']} ms/step median {d['ms_per_step_median']}", flush=True)
PY
}
for kf in 0 1; do
  AINP_NTCF_KFIRST=$kf timeout -k 10 120 python tools/bn_probe.py 10 > "$OUT/bn_probe_kf$kf.log" 2>&1 || exit 1
  echo "-- kfirst $kf"; grep -v amdgpu.ids "$OUT/bn_probe_kf$kf.log"
done
for rep in 1 2 3; do
  run c2 kfirst_$rep AINP_NTCF_KFIRST=1 || exit 1
  run c2 base_$rep AINP_DEFER_LIFO=0 || exit 1
  run c2 lifo_$rep AINP_DEFER_LIFO=1 || exit 1
  run c2 joint_$rep AINP_PROJ_JOINT=1 || exit 1
done
for rep in 1 2; do
  run c3 base_$rep AINP_DEFER_LIFO=0 || exit 1
  run c3 lifo_$rep AINP_DEFER_LIFO=1 || exit 1
done
echo "all steps ok"
