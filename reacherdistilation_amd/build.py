"""Build the native library in-tree: reacherdistilation_amd/libreacher.so (gfx950).

hipcc compiles each HIP / C++ source to an object (in parallel), then links the shared
object; nothing is JIT-compiled at import time and nothing goes to a cache outside the repo,
so the .so travels with the repo snapshot to the GPU box.

The product build has no run-time knobs: diagnostic and ablation paths (the consumer-side
env step, forced group sizes, the LSTM's per-step path selection for timing, ...) exist only
in `build_variant` builds, selected by -D macros.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libreacher.so")
OBJ = os.path.join(HERE, "build")
ARCH = os.environ.get("RD_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

# -O3; keep IEEE f32 semantics (no -ffast-math): parity tolerances are stated for it.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Werror",
          "-Wno-unused-function", "-munsafe-fp-atomics"]
LDFLAGS = ["-shared", f"--offload-arch={ARCH}", "-ldl"]
# Per-source flags.  distill.hip (the fused rollout) is compiled without SLP vectorisation: the
# SLP pass packed the producer's dW3 / db3 accumulators into v_pk_fma_f32 / v_pk_add_f32 at the
# tile loop's latch, whose operands the next tile's first LDS loads overwrite; on gfx950 a
# packed-f32 op queued behind MFMAs can read its operands after such a load landed, and lanes
# 48-63 of gw3b came out different run to run (DESIGN.md §3 "PKWAR", scripts/isa/hazards.py).
# Round 6 also unpacked the explicit f32x2 tanh / split pairs, so no rollout kernel contains a
# packed-f32 op at all.  ppo.hip: its minibatch kernel keeps 38 gradient sums per thread across
# tiles, and its SLP build had loads 14-46 instructions behind unread packed accumulators.
# student_mlp.hip / student_lstm.hip: their SLP builds had the same pattern (PKWAR hits in the
# reference student's kernel and reduce+Adam, the LSTM's BPTT, head and reduce kernels); every
# product source is now scanned for it (tests/test_product_hygiene.py).
NO_SLP = ["-fno-slp-vectorize"]
SRC_FLAGS = {"distill.hip": NO_SLP, "ppo.hip": NO_SLP, "student_mlp.hip": NO_SLP, "student_lstm.hip": NO_SLP}


def src_flags(path):
    return SRC_FLAGS.get(os.path.basename(path), [])
FLAGS = CFLAGS + LDFLAGS   # one-command form (resource_usage, scripts)


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


def _jobs():
    return max(1, min(len(sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))


def _link(out, opts=(), verbose=True):
    """Compile every source with `opts` in parallel, link `out` (atomically replaced)."""
    tag = os.path.splitext(os.path.basename(out))[0]
    odir = os.path.join(OBJ, tag)
    os.makedirs(odir, exist_ok=True)
    srcs = sources()
    objs = [os.path.join(odir, os.path.basename(s) + ".o") for s in srcs]

    def cc(pair):
        s, o = pair
        cmd = [HIPCC, *CFLAGS, *src_flags(s), *opts, "-c", "-o", o, s]
        r = subprocess.run(cmd, capture_output=True, text=True)
        return cmd, r

    with ThreadPoolExecutor(_jobs()) as ex:
        results = list(ex.map(cc, zip(srcs, objs)))
    for cmd, r in results:
        if verbose:
            print(" ".join(cmd), flush=True)
        if r.returncode:
            sys.stderr.write(r.stdout + r.stderr)
            raise subprocess.CalledProcessError(r.returncode, cmd)
    cmd = [HIPCC, *LDFLAGS, "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, verbose: bool = True, extra=()):
    if not force and up_to_date():
        return LIB
    return _link(LIB, tuple(extra), verbose)


def resource_usage():
    """Print per-kernel VGPR/SGPR/LDS/occupancy (hipcc -Rpass-analysis)."""
    for s in sources():
        subprocess.call([HIPCC, *CFLAGS, *src_flags(s), "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null", s])


def build_stamps():
    """Diagnostic build with per-wave phase stamps (scripts/stamps.py); never the product."""
    return _link(os.path.join(HERE, "libreacher_stamps.so"), ("-DRD_STAMPS",))


def build_variant(name, *defines):
    """Diagnostic build as libreacher_<name>.so; never the product.  Macros: RD_STAMPS,
    RD_MFMA_SRCC_FENCE (every f32 MFMA group of the rollout SrcC-fenced), or a compiler flag.
    The rejected schedule / ablation variants are kept as profiles/r04_removed_diagnostic_variants.diff
    (rollout) and profiles/r05_removed_diagnostic_variants.diff (LSTM, GEMM, PPO, env, reference
    student)."""
    opts = tuple(d if d.startswith("-") else f"-D{d}" for d in defines)
    return _link(os.path.join(HERE, f"libreacher_{name}.so"), opts)


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
