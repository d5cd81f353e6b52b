"""Scratch (private segment) of the shipped kernels, read on the CPU from the
in-tree liblnw.so's gfx950 code object metadata (llvm-objcopy, the offload
bundler, llvm-readelf --notes).

Round 6 measured what scratch costs these kernels: a launch-time register
preload that put 52 B per lane of scratch into the contact variants made melee
2.3-3 us slower, and a restructured small-workgroup path with 56 B ran the
8 192-env shard 1.8 us slower (small shards). The kernels that carry
the bench workloads must stay scratch-free; the small-shard kernel's 28 B (its
launch-time counter loads, measured faster with them) is pinned so that growth
shows up here, and so is the policy kernel's 20 B (its 64-bit row addresses
no longer live across the conv head: 28 -> 20 B, 3 us faster).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "littoral-naval-warfare-marl_amd", "lnw", "liblnw.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# mangled-name fragment -> largest scratch allowed (bytes per lane)
LIMITS = {
    "step_kernelILi4ELi4ELb0ELb0ELi4ELb0E": 0,   # headline: units kernel
    "step_kernelILi4ELi4ELb1ELb0ELi1ELb0E": 0,   # melee: contact variant
    "step_kernelILi4ELi4ELb1ELb0ELi1ELb1E": 0,   # config 5's step: contact, phase S by side
    "step_kernelILi4ELi4ELb0ELb0ELi1ELb0E": 28,  # small shards (config 2, config 3 at N = 8)
    "step_group_kernel": 0,                     # config 4
    "policy_act_kernel": 20,                    # config 5's policy (3 spilled 64-bit values;
                                                #  28 -> 20 B took 3 us off it, round 6)
    "rollout_post_kernel": 0,                   # config 5's critic
    "observe_kernelILi4ELi4ELb1E": 0,           # config 5's observe (contact variant)
}


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


def kernel_scratch(lib, tmp):
    """{kernel name: private segment bytes per lane} over every code object in
    the library's .hip_fatbin (one offload bundle per translation unit)."""
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib,
                    os.path.join(tmp, "host.so")], check=True, capture_output=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = {}
    for n, a in enumerate(starts):
        b = starts[n + 1] if n + 1 < len(starts) else len(data)
        part, co = os.path.join(tmp, f"b{n}.bin"), os.path.join(tmp, f"co{n}.o")
        with open(part, "wb") as f:
            f.write(data[a:b])
        subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s*\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
                continue
            m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
            if m and name:
                out[name] = int(m.group(1))
                name = None
    return out


@pytest.mark.skipif(not os.path.exists(LIB), reason="liblnw.so not built")
@pytest.mark.skipif(not (_tool("llvm-objcopy") and _tool("clang-offload-bundler") and _tool("llvm-readelf")),
                    reason="ROCm LLVM tools not found")
def test_bench_kernels_scratch(tmp_path):
    sc = kernel_scratch(LIB, str(tmp_path))
    assert sc, "no kernel metadata found"
    for frag, limit in LIMITS.items():
        hits = {k: v for k, v in sc.items() if frag in k}
        assert hits, f"kernel {frag} not in liblnw.so"
        for k, v in hits.items():
            assert v <= limit, f"{k}: {v} B/lane of scratch (limit {limit})"
