#!/bin/bash
# quick register/occupancy check of the rmsc03 kernels (device-only compile)
cd "$(dirname "$0")/../marl-optimal-execution_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -mllvm -structurizecfg-skip-uniform-regions -DMXA_ONLY_RMSC03 --cuda-device-only -c \
  -Icsrc -I../include csrc/mxa_api.hip -o /tmp/mxa_dev.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
  | grep -E "error|Function Name|VGPRs|AGPRs|SGPRs|Scratch|Occupancy|LDS" | grep -v "^ *[0-9]* |"
