#!/bin/bash
# GAN-side GPU pass: the GAN kernel/model parity tests, the GAN bench and a
# rocprofv3 kernel trace of it.  Each step has its own limit; stops at the first failure.
#   gpurun -- bash tools/gan_check.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-gan_check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gan or im2col or conv_gen or pconv or sn_ or vgg or disc" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --workload gan > "$OUT/bench_gan.json" 2>&1 || exit 1
tail -1 "$OUT/bench_gan.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d "$OUT/prof" -o run -- \
  python3 bench.py --workload gan --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit 1
echo ok
