#!/bin/bash
# Build the GEMM structure lab against the in-tree libainp.so.
set -e
cd "$(dirname "$0")"
hipcc -O3 -std=c++17 --offload-arch=gfx950 gemm_lab.hip -o gemm_lab \
  -L../ml-audio-inpainting_amd/ainp -lainp -Wl,-rpath,'$ORIGIN/../ml-audio-inpainting_amd/ainp' "$@"
