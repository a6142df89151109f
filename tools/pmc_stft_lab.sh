#!/bin/bash
# SQ counter passes over the STFT lab's candidate kernel alone (tools/stft_lab.hip, arg b).
#   gpurun -- bash tools/pmc_stft_lab.sh <binary> <tag>
set -o pipefail
BIN=${1:-./tools/stft_lab3}
OUT=gpurun_out/${2:-pmc_stft_lab}
MODE=${3:-b}
GRID=${4:-256}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -f csv -d "$OUT/sq1" -o run -- "$BIN" $MODE $GRID \
  > "$OUT/sq1.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
  SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES -f csv -d "$OUT/sq2" -o run -- "$BIN" $MODE $GRID > "$OUT/sq2.log" 2>&1 || exit 1
for p in sq1 sq2; do
  f=$(find "$OUT/$p" -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, collections, sys
d = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    k = (int(r["Dispatch_Id"]), r["Kernel_Name"][:40])
    d.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    d[k]["dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    d[k]["vgpr"] = r["VGPR_Count"]
for k, v in list(d.items())[-2:]:
    print(k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items()})
PY
done
