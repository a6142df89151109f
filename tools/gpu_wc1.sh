#!/bin/bash
# Cout=1 weight gradient (ainp_wgrad_cout1): GAN + D-backward parity tests,
# C4 bf16 A/B against im2col16 + GEMM (AINP_WGRAD_COUT1=0; the second digit
# was AINP_COUT1_NHWC16, the channel-last Cout=1 conv of run wc4, since
# dropped), GAN step kernel stats.
set -o pipefail
OUT=gpurun_out/${1:-wc1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_dconv16.py -x -v --timeout 120 \
  --timeout-method thread > "$OUT/pytest_gan.log" 2>&1 || { tail -30 "$OUT/pytest_gan.log"; exit 1; }
tail -1 "$OUT/pytest_gan.log"
for v in ${AB:-00 10 00 10}; do
  AINP_WGRAD_COUT1=${v:0:1} AINP_COUT1_NHWC16=${v:1:1} timeout -k 10 300 python bench.py --workload gan \
    --dtype bf16 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err" || { tail -5 "$OUT/c4_$v.err"; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c4_$v.json').read().strip().splitlines()[-1]);print('wgrad_cout1,cout1_nhwc16=$v',d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/gan_bf16" -o run -- \
  python3 tools/step_prof.py --workload gan --steps 6 --dtype bf16 > "$OUT/gan_prof.log" 2>&1 || { tail -5 "$OUT/gan_prof.log"; exit 1; }
echo "all ok"
