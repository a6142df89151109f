#!/bin/bash
# 2-rank data-parallel rehearsal on the box's one GPU over gloo (host-staged
# collectives; says nothing about RCCL/xGMI): the bench's dp block
# (all-reduce alone, compute-only step, overlap) for the C2 fp32 and the bf16
# C3-shape steps, and the 2-rank GPU DP tests.
set -o pipefail
OUT=gpurun_out/${1:-dp2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_dist.log" 2>&1; rc=$?
tail -1 "$OUT/pytest_dist.log"; [ $rc -eq 0 ] || exit 1
for dt in fp32 bf16; do
  AINP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
    --no-graph --dtype $dt > "$OUT/dp2_gloo_$dt.json" 2> "$OUT/dp2_gloo_$dt.err" || exit 1
  tail -1 "$OUT/dp2_gloo_$dt.json" | cut -c1-200
done
echo "all ok"
