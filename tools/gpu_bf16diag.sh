#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-bf16diag}
mkdir -p "$OUT"
for v in fp32 bf16 bf16_staged_l0 conv_bf16_only gemm_bf16_only; do
  timeout -k 10 120 python tools/bf16_grad_diag.py $v > "$OUT/$v.log" 2>&1 || { echo "fail $v"; cat "$OUT/$v.log" | tail -5; exit 1; }
  cat "$OUT/$v.log"
done
AINP_B16_PROJ_SPLIT=1 timeout -k 10 120 python tools/bf16_grad_diag.py bf16 > "$OUT/bf16_nosplit.log" 2>&1 && cat "$OUT/bf16_nosplit.log"
