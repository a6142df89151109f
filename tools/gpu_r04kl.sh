#!/bin/bash
# r04k (bf16 pre-BN storage parity + C3 A/B) then r04l (deferred-gradient
# order A/B) in one call.
bash tools/gpu_r04k.sh "${1:-r04kl}" && bash tools/gpu_r04l.sh "${1:-r04kl}"
