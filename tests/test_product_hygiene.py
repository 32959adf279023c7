"""Host-side (no GPU) checks that the PRODUCT library is the product (VERDICT r2, next-round
item 2): no run-time knobs, no diagnostic kernels, the ctypes mirrors match the C headers
byte for byte, and the bench's headline mode is the library's default mode.

- libreacher.so imports no getenv: every measurement-only switch (RDD_PHYS, RDD_GROUP_ENVS,
  RDM_ROWS, RDL_PR_DBG) exists only in build_variant builds (-DRD_DIAG_KNOBS / -DRD_CP_VARIANT);
  the tests' path selections are config fields (rdd_config.group_envs, rdl_config.kernels).
- The consumer-side env step is instantiated only for the bf16 student (rollout_kernel<true, *,
  true>), whose f32 MFMAs (the teacher's) are SrcC-fenced; the f32 student's consumer-side step
  (its consumer runs 80 unfenced f32 MFMAs per tile) exists only in diagnostic
  builds.
- Statically, in the product's ISA no LDS / global load is issued into a register that an
  in-flight f32 MFMA (8 passes) still reads as SrcC: every such load comes >= 10 wait states
  after the MFMA, i.e. after it completed -- the pattern that made the unfenced consumer-side
  step lose loaded values in lanes 48-63 (scripts/isa/hazards.py, profiles/r03_srcc_probe_*.txt).
  The split kernels (the default mode) have no f32 MFMA followed by such a load at all.
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from tests.conftest import ROOT


@pytest.fixture(scope="module")
def libpath():
    from reacherdistilation_amd import _native, build
    build.build(verbose=False)
    _native.load()
    return build.LIB


def test_product_library_reads_no_environment(libpath):
    out = subprocess.run(["nm", "-D", "--undefined-only", libpath], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}
    assert not {"getenv", "secure_getenv", "__secure_getenv"} & syms


def test_consumer_side_step_only_for_the_bf16_student(libpath):
    blob = open(libpath, "rb").read()
    names = set(re.findall(rb"rollout_kernelILb[01]ELb[01]ELb[01]E", blob))
    assert names, "rollout_kernel instantiations not found in the offload bundle"
    # <bf16 student, f32 mode, consumer-side step>: f32 student -> producer-side, bf16 -> consumer-side
    assert names == {b"rollout_kernelILb0ELb0ELb0E", b"rollout_kernelILb0ELb1ELb0E",
                     b"rollout_kernelILb1ELb0ELb1E", b"rollout_kernelILb1ELb1ELb1E"}, sorted(names)


def test_no_load_into_an_inflight_f32_mfma_srcc():
    """The product's rollout kernels, compiled to ISA here: every LDS / global load whose
    destination is the SrcC of an earlier v_mfma_f32_16x16x4_f32 issues >= 10 wait states after
    it, i.e. after the MFMA completed (the compiler's RAW wait for an 8-pass result, NumPasses +
    2; ROCm 7.2 itself only keeps 3-5 for this WAR).  In the split kernels no load follows an
    f32 MFMA into its SrcC within the scan window at all (their f32 MFMAs are dW1 only)."""
    import importlib.util
    from reacherdistilation_amd import build
    out = os.path.join(ROOT, "oracle", "_build", "distill_isa.s")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([build.HIPCC, "-O3", "-std=c++17", f"--offload-arch={build.ARCH}", "-munsafe-fp-atomics",
                    "--cuda-device-only", "-S", "-o", out, os.path.join(build.CSRC, "distill.hip")],
                   check=True, capture_output=True)
    spec = importlib.util.spec_from_file_location("hz", os.path.join(ROOT, "scripts", "isa", "hazards.py"))
    hz = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(hz)
    for sym, split in (("rollout_kernelILb0ELb0ELb0E", False), ("rollout_kernelILb0ELb1ELb0E", True),
                       ("rollout_kernelILb1ELb0ELb1E", False), ("rollout_kernelILb1ELb1ELb1E", True)):
        hits = [h for h in hz.scan(out, sym, 40)[0] if h[0] == "WARc" and "16x16x4" in h[4]
                and h[6].split()[0].startswith(("ds_read", "global_load", "buffer_load"))]
        assert all(h[1] >= 10 for h in hits), (sym, [h[:6] for h in hits if h[1] < 10][:5])
        if split:
            assert not hits, (sym, [h[:6] for h in hits][:5])


def _c_layout(struct, header, fields):
    """sizeof and offsetof of a header struct, compiled with gcc from the header itself."""
    body = "\n".join(f'printf("{f} %zu\\n", offsetof({struct}, {f}));' for f in fields)
    src = (f'#include <stddef.h>\n#include <stdio.h>\n#include "{header}"\n'
           f'int main(void) {{ printf("sizeof %zu\\n", sizeof({struct})); {body} return 0; }}\n')
    d = os.path.join(ROOT, "oracle", "_build")
    os.makedirs(d, exist_ok=True)
    c, exe = os.path.join(d, f"layout_{struct}.c"), os.path.join(d, f"layout_{struct}")
    with open(c, "w") as fh:
        fh.write(src)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c], check=True)
    res = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    return {k: int(v) for k, v in (ln.split() for ln in res.splitlines())}


@pytest.mark.parametrize("mod,cls,struct,header", [
    ("reacherdistilation_amd.distill", "RddConfig", "rdd_config", "reacher_distill.h"),
    ("reacherdistilation_amd.student_lstm", "RdlConfig", "rdl_config", "reacher_student_lstm.h"),
    ("reacherdistilation_amd.student_mlp", "RdmConfig", "rdm_config", "reacher_student_mlp.h"),
    ("reacherdistilation_amd.ppo", "RdpConfig", "rdp_config", "reacher_ppo.h"),
])
def test_ctypes_configs_match_the_headers(mod, cls, struct, header):
    import importlib
    C = getattr(importlib.import_module(mod), cls)
    fields = [f[0] for f in C._fields_]
    c = _c_layout(struct, header, fields)
    assert c["sizeof"] == ctypes.sizeof(C)
    for f in fields:
        assert c[f] == getattr(C, f).offset, f
    # every member of the C struct is mirrored (no field missing on the Python side)
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    body = re.search(r"typedef struct \{(.*?)\}\s*" + struct + ";", txt, re.S).group(1)
    names = re.findall(r"(\w+)\s*(?:,|;)", body)
    assert sorted(names) == sorted(fields)


def test_bench_headline_mode_is_the_library_default(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    from reacherdistilation_amd.distill import DistillConfig
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse()
    assert (args.f32_mode == "split") == DistillConfig().f32_split
