#!/bin/bash
# resource usage of one HIP translation unit: name VGPR AGPR scratch occupancy
cd /root/repo/slam-uwv_kalman_filters_amd
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-result -mllvm -disable-machine-licm -mllvm -amdgpu-mfma-vgpr-form $2 -c ${1:-csrc/uwvk_psp_k.hip} -o /tmp/ru.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "error|Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy" | paste - - - - - | sed 's/remark://g; s/\[-Rpass-analysis=kernel-resource-usage\]//g; s/csrc\/[a-z_]*.hip:[0-9]*:[0-9]*://g; s/Function Name: _ZN4uwvk3psp//' | awk '{print $1, $3, $5, $8, $11}'
