#!/bin/bash
# Stand-alone x6r launches (tools/roofline_probe.py: the layer-0 projection
# and the backward pair) under two environments; per-launch average duration
# from rocprofv3 --kernel-trace --stats.
#   gpurun -- bash tools/x6r_ab.sh <tag> "ENV_A" "ENV_B"
set -o pipefail
OUT=gpurun_out/${1:?tag}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in A B; do
  if [ $v = A ]; then envs=${2//,/ }; else envs=${3//,/ }; fi
  for mode in fp32 pair; do
    env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${v}_$mode" -o run -- \
      python3 tools/roofline_probe.py 10 $mode > "$OUT/${v}_$mode.log" 2>&1 || exit 1
    python3 - "$OUT/${v}_$mode/run_kernel_stats.csv" "$v $mode ($envs)" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm_x6r" in r["Name"]:
        print(sys.argv[2], "calls", r["Calls"], "avg ms %.3f" % (float(r["AverageNs"]) / 1e6),
              "min ms %.3f" % (float(r["MinNs"]) / 1e6))
PY
  done
done
echo "all steps ok"
