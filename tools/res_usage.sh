#!/bin/bash
# Register / scratch usage of the v2 step kernel instantiations (compile-only, host side).
# usage: tools/res_usage.sh [source]   (default csrc/ch_step.hip)
SRC=${1:-rl-cattle-herding_amd/csrc/ch_step.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Iinclude \
  --cuda-device-only -c "$SRC" -o /tmp/res_usage.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs:" |
  sed -E 's/.*remark: //' | paste - - - - - - | grep -E "${FILTER:-k_step2}" | sed -E 's/\s+/ /g'
