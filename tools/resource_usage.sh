# Per-kernel register / scratch / LDS usage of liblnw's step kernels (gfx950),
# from the compiler's kernel-resource-usage remarks: bash tools/resource_usage.sh
cd "$(dirname "$0")/.." || exit 1
C=littoral-naval-warfare-marl_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -Iinclude -I$C --cuda-device-only -c $C/lnw_kernels.hip -o /tmp/lnw_ru.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" \
  | sed -e 's/.*remark: //' | paste - - - - - - | sed -e 's/\[-Rpass-analysis=kernel-resource-usage\]//g' | grep -E "step_kernel|step_group"
