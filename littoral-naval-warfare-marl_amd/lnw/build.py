"""Build liblnw.so in-tree for gfx950 with hipcc (no JIT cache, no CPU path).

-ffp-contract=off keeps every float/double operation un-fused so the kernels
round exactly like CPython/NumPy (the reference); see DESIGN.md "Numerics".
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "liblnw.so")
# diagnostics build: LNW_DEBUG_SKIP section skips (results change) and the
# group kernel's section timers; never loaded unless LNW_LIB names it
DIAG_OUT = os.path.join(HERE, "liblnw_diag.so")
DIAG_DEFINES = ("LNW_DIAG", "LNW_GROUP_PROF")
SOURCES = [os.path.join(CSRC, "lnw_kernels.hip"), os.path.join(CSRC, "lnw_actor.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "lnw_device.h"), os.path.join(CSRC, "lnw_quiet.inc"),
                  os.path.join(CSRC, "lnw_group.inc"),
                  os.path.join(INCLUDE, "lnw.h")]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def flags(arch="gfx950"):
    return [f"--offload-arch={arch}", "-O3", "-std=c++17", "-ffp-contract=off",
            "-fno-gpu-flush-denormals-to-zero", "-fPIC", "-shared", f"-I{INCLUDE}", f"-I{CSRC}"]


def source_digest():
    """SHA-256 over the compiler flags and every source liblnw.so is built
    from: identifies the kernel code a measurement was taken on (hipcc's output
    bytes differ between otherwise identical builds)."""
    import hashlib
    # flags without the include paths (the tree's location differs between machines)
    h = hashlib.sha256(" ".join(f for f in flags() if not f.startswith("-I")).encode())
    for d in DEPS:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build(force=False, verbose=False, out=OUT, defines=()):
    """liblnw.so (or a diagnostics variant at `out` built with -D`defines`)."""
    if not force and os.path.exists(out):
        t = os.path.getmtime(out)
        if all(os.path.getmtime(d) <= t for d in DEPS):
            return out
    cmd = [hipcc()] + flags() + [f"-D{d}" for d in defines] + SOURCES + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed building liblnw.so")
    os.replace(out + ".tmp", out)
    return out


def build_diag(force=False, verbose=False):
    return build(force=force, verbose=verbose, out=DIAG_OUT, defines=DIAG_DEFINES)


if __name__ == "__main__":
    if "--diag" in sys.argv:
        print(build_diag(force="--force" in sys.argv, verbose=True))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
