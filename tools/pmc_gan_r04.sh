#!/bin/bash
# rocprofv3 FETCH_SIZE / WRITE_SIZE passes (one counter per run) over the GAN
# bench's two roofline kernels at both GAN shapes, on the in-step operands
# (tools/roofline_probe_gan.py): the final PartialConv2d (65 -> 64 at
# 384 x 640 / 1024) and U-Net decoder block 3 (768 -> 256 at 48 x 80 / 128).
#   gpurun -- bash tools/pmc_gan_r04.sh <tag>
set -o pipefail
TAG=${1:-pmc_gan_r04}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <dir> <counter> <clip_s> <which>
  echo "== $(date +%T) pmc $1: $2"
  timeout -s KILL 120 rocprofv3 --pmc "$2" -f csv -d "$OUT/$1" -o run -- \
    python3 tools/roofline_probe_gan.py 5 bf16 "$3" "$4" > "$OUT/$1.log" 2>&1
  local rc=$?
  echo "   rc=$rc"
  return $rc
}
for cs in 5 8; do
  W=$([ $cs = 8 ] && echo 1024 || echo 640)
  for which in final wide; do
    d=${which}_c$cs
    mkdir -p "$OUT/$d"
    pass "$d/fetch" FETCH_SIZE $cs $which || exit 1
    pass "$d/write" WRITE_SIZE $cs $which || exit 1
    if [ $which = final ]; then
      # x0 bf16 NHWC 8x192x(W/2)x64 + expanded skip rows 8x384xW x 32 bf16 + ratio fp32
      # + out fp32 8x64x384xW + weights 64x608 bf16
      ALG=$(( 2*8*192*(W/2)*64 + 2*8*384*W*32 + 4*8*384*W + 4*8*64*384*W + 2*64*608 ))
      KN="conv_gen_nhwc16_kernel<64"
    else
      # src0 bf16 NHWC 8x24x(W/16)x512 (read at its own resolution) + skip 8x48x(W/8)x256
      # + ratio fp32 8x48x(W/8) + out fp32 8x256x48x(W/8) + weights 256x6912 bf16
      ALG=$(( 2*8*24*(W/16)*512 + 2*8*48*(W/8)*256 + 4*8*48*(W/8) + 4*8*256*48*(W/8) + 2*256*6912 ))
      KN="conv_gen_nhwc16_wide_kernel<256"
    fi
    # the probe's G forward launches the same kernels first: the last 4 of its
    # 5 launches are the measured ones
    python3 tools/traffic_json.py "$OUT/$d" "$KN" $ALG \
      "tools/pmc_gan_r04.sh: tools/roofline_probe_gan.py 5 bf16 $cs $which (in-step operands)" 4 \
      > "$OUT/$d/traffic.json" && cat "$OUT/$d/traffic.json" || exit 1
  done
done
echo "all passes ok"
