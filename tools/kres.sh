#!/bin/bash
# Register / LDS / scratch usage of the rollout kernel variants (compile only,
# CPU container):  tools/kres.sh [-D...]
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -c -O3 -std=c++17 -fPIC -Wno-pass-failed \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -Xarch_device -freciprocal-math -Xarch_device -fapprox-func \
  -mllvm -simplifycfg-sink-common=false -Xarch_device -fno-slp-vectorize -Xarch_device -fassociative-math \
  -Xarch_device -fno-signed-zeros -Xarch_device -fno-trapping-math "$@" \
  -Rpass-analysis=kernel-resource-usage -o /tmp/kres.o manipulator_mujoco_amd/csrc/rollout.hip 2>&1 |
  grep -A12 "Function Name: .*rollout_kernel" | grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size|SGPRs:" |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
