#!/bin/bash
# ab7 (Cout=1 strip kernel A/B) then the wide-conv PMC passes.
set -o pipefail
bash tools/gpu_ab7.sh "${1:-ab7}" || exit 1
bash tools/pmc_wide.sh "${2:-pmc_wide}" || exit 1
