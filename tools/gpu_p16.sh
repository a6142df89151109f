#!/bin/bash
# bf16 layer-0 backward on ONE 256x256 grid (ainp_gemm_bf16nt_pair): GEMM and
# (AINP_L0_PAIR16 / ainp_gemm_bf16nt_pair were the experiment of profiles/r03_p16_summary.txt; dropped.)
# CNNBLSTM GPU tests, C3-shape bf16 A/B against the two-stream g16 launches
# (AINP_L0_PAIR16=0), bf16 step kernel stats.
set -o pipefail
OUT=gpurun_out/${1:-p16}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 200 \
  --timeout-method thread -k "bf16nt or bf16 or model" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in ${AB:-0 1 0 1}; do
  AINP_L0_PAIR16=$v timeout -k 10 300 python bench.py --dtype bf16 --steps 30 --warmup 5 --no-cpu-baseline \
    > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err" || { tail -5 "$OUT/c3_$v.err"; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c3_$v.json').read().strip().splitlines()[-1]);print('pair16=$v',d['ms_per_step'],d['ms_per_step_median'],d.get('roofline_l0_bwd',{}).get('avg_launch_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/cnn_bf16" -o run -- \
  python3 tools/step_prof.py --steps 10 --dtype bf16 > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 1; }
echo "all ok"
