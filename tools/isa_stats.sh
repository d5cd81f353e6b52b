# Instruction mix and scratch traffic of one kernel in liblnw's device code:
#   bash tools/isa_stats.sh step_group_kernel
cd "$(dirname "$0")/.." || exit 1
C=littoral-naval-warfare-marl_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -Iinclude -I${SRC:-$C} --cuda-device-only -c ${SRC:-$C}/lnw_kernels.hip -o /tmp/lnw_isa.o 2>/dev/null || exit 1
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/lnw_isa.o \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/lnw_isa_dev.o || exit 1
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 /tmp/lnw_isa_dev.o > /tmp/lnw_isa.txt
python3 - "$1" <<'PY'
import collections, re, sys
s = open('/tmp/lnw_isa.txt').read()
m = re.search(r'\n[0-9a-f]+ <([^>]*' + sys.argv[1] + r'[^>]*)>:\n', s)
i = m.end()
n = re.search(r'\n[0-9a-f]+ <[^>]+>:\n', s[i:])
body = [l.strip().split()[0] for l in s[i:i + (n.start() if n else len(s))].split('\n') if l.strip()]
c = collections.Counter(body)
print(m.group(1)[:60], len(body), 'instructions')
for k in ('scratch_load_dword', 'scratch_store_dword', 'scratch_load_dwordx2', 'scratch_store_dwordx2',
          'scratch_load_dwordx4', 'scratch_store_dwordx4', 'v_readlane_b32', 'v_writelane_b32',
          'v_add_f64', 'v_mul_f64', 'v_fma_f64', 'global_load_dword', 'ds_read_b64'):
    print(f'  {k}: {c.get(k, 0)}')
PY
