#!/bin/bash
# Round-3 GPU pass (b): gpu_r03.sh + GAN C4 bf16 / C5 bf16 benches (C5 line
# carries the ISTFT / Griffin-Lim timings).
#   gpurun -- bash tools/gpu_r03b.sh <tag> [prof|noprof] [pytest -k expr]
set -o pipefail
TAG=${1:-r03b}
bash tools/gpu_r03.sh "$TAG" "${2:-noprof}" "$3" || exit 1
OUT=gpurun_out/$TAG
echo "== $(date +%T) gan c4 bf16"
timeout -k 10 300 python bench.py --workload gan --dtype bf16 --no-cpu-baseline > "$OUT/bench_gan_c4_bf16.json" 2>&1 || exit 1
tail -1 "$OUT/bench_gan_c4_bf16.json" | cut -c1-300
echo "== $(date +%T) gan c5 bf16"
timeout -k 10 300 python bench.py --workload gan --clip-s 8 --dtype bf16 --no-cpu-baseline > "$OUT/bench_gan_c5.json" 2>&1 || exit 1
tail -1 "$OUT/bench_gan_c5.json" | cut -c1-300
echo "all b steps ok"
