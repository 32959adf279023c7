"""Build the native library in-tree: reacherdistilation_amd/libreacher.so (gfx950).

hipcc compiles the HIP kernels and the C ABI straight to a shared object; nothing is
JIT-compiled at import time and nothing goes to a cache outside the repo, so the .so
travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libreacher.so")
ARCH = os.environ.get("RD_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# -O3; keep IEEE f32 semantics (no -ffast-math): parity tolerances are stated for it.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-Wall",
         "-Wno-unused-function", "-Werror=return-type", "-munsafe-fp-atomics", "-ldl"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + \
        sorted(glob.glob(os.path.join(HERE, "..", "include", "*.h")))


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in deps())


def build(force: bool = False, verbose: bool = True, extra=()):
    if not force and up_to_date():
        return LIB
    cmd = [HIPCC, *FLAGS, *extra, "-o", LIB + ".tmp", *sources()]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def resource_usage():
    """Print per-kernel VGPR/SGPR/LDS/occupancy (hipcc -Rpass-analysis)."""
    cmd = [HIPCC, *FLAGS, "-Rpass-analysis=kernel-resource-usage", "-o", "/dev/null", *sources()]
    subprocess.call(cmd)


def build_stamps():
    """Diagnostic build with per-wave phase stamps (scripts/stamps.py); never the product."""
    out = os.path.join(HERE, "libreacher_stamps.so")
    subprocess.check_call([HIPCC, *FLAGS, "-DRD_STAMPS", "-o", out, *sources()])
    return out


def build_variant(name, *defines):
    """Diagnostic/ablation build (e.g. RD_ABL_TANH, or a compiler flag such as
    -fno-slp-vectorize) as libreacher_<name>.so; never the product."""
    out = os.path.join(HERE, f"libreacher_{name}.so")
    opts = [d if d.startswith("-") else f"-D{d}" for d in defines]
    subprocess.check_call([HIPCC, *FLAGS, *opts, "-o", out, *sources()])
    return out


if __name__ == "__main__":
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        build_variant(sys.argv[i + 1], *sys.argv[i + 2:])
    elif "--usage" in sys.argv:
        resource_usage()
    elif "--stamps" in sys.argv:
        build_stamps()
    else:
        build(force="--force" in sys.argv)
