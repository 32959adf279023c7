"""Host-side (no GPU) checks that the PRODUCT library is the product (VERDICT r2, next-round
item 2): no run-time knobs, no diagnostic kernels, the ctypes mirrors match the C headers
byte for byte, and the bench's headline mode is the library's default mode.

- libreacher.so imports no getenv: the tests' path selections are config fields
  (rdd_config.group_envs, rdl_config.kernels).  distill.hip keeps two diagnostic macros
  (RD_STAMPS, RD_MFMA_SRCC_FENCE), the other sources none; the rejected variants live in
  profiles/*.diff.
- The consumer-side env step is instantiated only for the bf16 student (rollout_kernel<true, *,
  true>), whose f32 MFMAs (the exact teacher's) are SrcC-fenced.
- Statically, in the product's ISA no LDS / global load is issued into a register that an
  in-flight f32 MFMA (8 passes) still reads as SrcC unless an instruction in between forced the
  MFMA to complete -- the pattern that made the unfenced consumer-side step lose loaded values in
  lanes 48-63 (scripts/isa/hazards.py scan_ldsrc, profiles/r03_srcc_probe_*.txt); and no load
  overwrites a source of an unread packed-f32 op (scan_pkwar), the rollout having none at all.
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
    names = set(re.findall(rb"rollout_kernelILb[01]ELb[01]ELb[01]ELi[0-9]ELb[01]E", blob))
    assert names, "rollout_kernel instantiations not found in the offload bundle"
    # <bf16 student, f32 mode, consumer-side step, MD, K steps per launch>: f32 student ->
    # producer-side, bf16 -> consumer-side; MD 1 (rows: no env step) -> no consumer-side step, no
    # teacher; MD 2 (helper pairs of a small batch) -> f32 student only; the K-step launches
    # (rdd_step_accum) -> teacher mode, producer-side step, both students
    assert names == {b"rollout_kernelILb0ELb0ELb0ELi0ELb0E", b"rollout_kernelILb0ELb1ELb0ELi0ELb0E",
                     b"rollout_kernelILb1ELb0ELb1ELi0ELb0E", b"rollout_kernelILb1ELb1ELb1ELi0ELb0E",
                     b"rollout_kernelILb0ELb0ELb0ELi1ELb0E", b"rollout_kernelILb0ELb1ELb0ELi1ELb0E",
                     b"rollout_kernelILb1ELb0ELb0ELi1ELb0E",
                     b"rollout_kernelILb0ELb0ELb0ELi2ELb0E", b"rollout_kernelILb0ELb1ELb0ELi2ELb0E",
                     b"rollout_kernelILb0ELb0ELb0ELi0ELb1E", b"rollout_kernelILb0ELb1ELb0ELi0ELb1E",
                     b"rollout_kernelILb1ELb0ELb0ELi0ELb1E", b"rollout_kernelILb1ELb1ELb0ELi0ELb1E"}, sorted(names)


def _hz():
    import importlib.util
    spec = importlib.util.spec_from_file_location("hz", os.path.join(ROOT, "scripts", "isa", "hazards.py"))
    hz = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(hz)
    return hz


@pytest.fixture(scope="module")
def product_isa():
    """Every .hip source of the product compiled to gfx950 ISA here (hipcc -S, the product's flags)."""
    from concurrent.futures import ThreadPoolExecutor
    from reacherdistilation_amd import build
    d = os.path.join(ROOT, "oracle", "_build", "isa")
    os.makedirs(d, exist_ok=True)
    srcs = sorted(f for f in os.listdir(build.CSRC) if f.endswith(".hip"))

    def cc(f):
        out = os.path.join(d, f[:-4] + ".s")
        subprocess.run([build.HIPCC, "-O3", "-std=c++17", f"--offload-arch={build.ARCH}", "-munsafe-fp-atomics",
                        *build.src_flags(f), "-Wno-unused-command-line-argument", "--cuda-device-only", "-S",
                        "-o", out, os.path.join(build.CSRC, f)], check=True, capture_output=True)
        return f, out

    with ThreadPoolExecutor(len(srcs)) as ex:
        return dict(ex.map(cc, srcs))


def test_no_load_into_an_inflight_f32_mfma_srcc(product_isa):
    """VERDICT r5 item 1 (LDSRC by interlock, no distance exemption): in every function of every
    product source, no LDS / global load writes a SrcC register of an exact-f32 MFMA
    (v_mfma_f32_16x16x4_f32, 8 passes) within its NP + 6 wait-state horizon unless an instruction
    in between forces that MFMA to complete (a VALU / memory read of its result, an MFMA reading it
    as SrcA/B, an interlocked VALU write of the SrcC registers) -- hazards.py scan_ldsrc.  The
    exact pair forward's per-site fences (distill.hip kPairFence) are what makes the exact-f32
    rollout instances pass; the split (default) and bf16 instances pass unfenced."""
    hz = _hz()
    bad, nf32 = {}, 0
    for src, path in product_isa.items():
        for name, code in hz.functions(path).items():
            nf32 += sum(1 for _, l in code if l.startswith("v_mfma_f32_16x16x4"))
            hits = hz.scan_ldsrc(code)
            if hits:
                bad[f"{src}:{name}"] = [h[:6] for h in hits[:3]]
    assert nf32 > 1000, nf32   # the scan saw the exact-f32 MFMAs (rollout, PPO, LSTM, reference student)
    assert not bad, bad


ROLLOUT_SYMS = ("rollout_kernelILb0ELb0ELb0ELi0ELb0E", "rollout_kernelILb0ELb1ELb0ELi0ELb0E",
                "rollout_kernelILb1ELb0ELb1ELi0ELb0E", "rollout_kernelILb1ELb1ELb1ELi0ELb0E",
                "rollout_kernelILb0ELb0ELb0ELi1ELb0E", "rollout_kernelILb0ELb1ELb0ELi1ELb0E",
                "rollout_kernelILb1ELb0ELb0ELi1ELb0E",
                "rollout_kernelILb0ELb0ELb0ELi2ELb0E", "rollout_kernelILb0ELb1ELb0ELi2ELb0E",
                "rollout_kernelILb0ELb0ELb0ELi0ELb1E", "rollout_kernelILb0ELb1ELb0ELi0ELb1E",
                "rollout_kernelILb1ELb0ELb0ELi0ELb1E", "rollout_kernelILb1ELb1ELb0ELi0ELb1E")


def test_no_packed_f32_op_in_the_rollout_and_no_pkwar_anywhere(product_isa):
    """PKWAR (scripts/isa/hazards.py), closed by construction:
    - the rollout kernels contain no packed-f32 instruction (v_pk_fma/mul/add_f32) at all: distill.hip
      is built without SLP and its tanh / operand splits / partial-row sums are scalar code;
    - in every function of every product source no LDS / global load overwrites a source of a
      packed-f32 op that nothing has read yet (scan_pkwar, no distance exemption): ppo.hip,
      student_mlp.hip and student_lstm.hip are built without SLP too (build.SRC_FLAGS)."""
    hz = _hz()
    fns = hz.functions(product_isa["distill.hip"])
    for sym in ROLLOUT_SYMS:
        name = next(n for n in fns if sym in n)
        pk = [(ln, l) for ln, l in fns[name] if l.startswith(hz.PK_F32)]
        assert not pk, (sym, pk[:5])
    bad = {}
    for src, path in product_isa.items():
        for name, code in hz.functions(path).items():
            hits = hz.scan_pkwar(code)
            if hits:
                bad[f"{src}:{name}"] = [h[:6] for h in hits[:3]]
    assert not bad, bad


def test_no_hazard_below_its_requirement_in_any_kernel(product_isa):
    """VERDICT r3 item 2 / ADVICE r3: every function of every .hip source (rollout, forward,
    reduce, env, reference student, LSTM, GEMM, PPO, xGMI), scanned along its control flow (loop
    back-edges included) for every class of scripts/isa/hazards.py -- loads into an in-flight
    MFMA's SrcC (f32: before completion), MFMA result reads/writes, MFMA-to-MFMA operands,
    VALU-written MFMA operands, VMEM store data overwritten before the store read it, v_permlane
    operands, transcendental results, VALU-written SGPRs used by VMEM: none below its
    requirement.  (Round 4 found and fenced two: the reference student's 64-row weight gradient,
    LDS loads 0-9 wait states into in-flight f32 SrcC, and the bf16 forward kernel's teacher.)"""
    hz = _hz()
    bad = {}
    nfn = 0
    for src, path in product_isa.items():
        for name, code in hz.functions(path).items():
            nfn += 1
            v = hz.violations(hz.scan_code(code, 40))
            if v:
                bad[f"{src}:{name}"] = [h[:6] for h in v[:3]]
    assert nfn >= 90, nfn
    assert not bad, bad


@pytest.mark.parametrize("kind,snippet", [
    ("LDSRC", ["v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[8:11]", "ds_read_b128 v[8:11], v6"]),
    ("LDSRC", ["v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[8:11]", "s_add_u32 s0, s0, 1",
               "s_cbranch_scc1 .LBB0_1", "s_endpgm", ".LBB0_1:", "global_load_dword v9, v[12:13], off"]),
    ("WARc", ["v_mfma_f32_16x16x32_bf16 v[0:3], v[4:7], v[12:15], v[8:11]", "v_mov_b32_e32 v8, 0"]),
    ("RAW", ["v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[0:3]", "s_nop 3", "v_add_f32_e32 v6, v0, v7"]),
    ("MRAW", ["v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[0:3]", "v_mfma_f32_16x16x4_f32 v[8:11], v0, v5, v[8:11]"]),
    ("VMFMA", ["v_add_f32_e32 v4, v5, v6", "v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[0:3]"]),
    ("STDATA", ["global_store_dwordx4 v[10:11], v[0:3], off nt", "v_mov_b32_e32 v2, 0"]),
    ("PERM", ["v_add_f32_e32 v1, v2, v3", "v_permlane32_swap_b32_e32 v1, v4"]),
    ("TRANS", ["v_exp_f32_e32 v1, v2", "v_add_f32_e32 v3, v1, v4"]),
    ("SGPRV", ["v_readfirstlane_b32 s4, v1", "global_load_dword v2, v3, s[4:5]"]),
])
def test_hazard_scanner_detects_each_class(kind, snippet):
    """Positive controls: one pair below the requirement per class (the second LDSRC case only
    through a taken branch) is reported; the same pair padded with s_nop 15 is not."""
    hz = _hz()
    code = [(i + 1, l) for i, l in enumerate(snippet)]
    assert kind in {h[0] for h in hz.violations(hz.scan_code(code, 40))}
    padded = [code[0], (0, "s_nop 15"), (0, "s_nop 15")] + code[1:]
    assert kind not in {h[0] for h in hz.violations(hz.scan_code(padded, 40))}


def test_distill_keeps_only_two_diagnostic_macros():
    """the rejected schedule / ablation variants live in
    profiles/r04_removed_diagnostic_variants.diff and profiles/r05_removed_diagnostic_variants.diff,
    not in the product sources: distill.hip keeps RD_STAMPS and RD_MFMA_SRCC_FENCE, the other
    sources no conditional compilation at all."""
    from reacherdistilation_amd import build
    for src in build.sources() + [os.path.join(build.CSRC, f) for f in os.listdir(build.CSRC) if f.endswith(".h")]:
        txt = open(src).read()
        macros = set(re.findall(r"^#\s*if(?:n?def)?\s+(?:defined\()?(\w+)", txt, re.M))
        allowed = {"RD_STAMPS", "RD_MFMA_SRCC_FENCE"} if src.endswith("distill.hip") else set()
        assert macros <= allowed, (os.path.basename(src), macros)


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


def test_interlock_scanners_positive_controls():
    """scan_ldsrc / scan_pkwar report a load into an in-flight exact-f32 MFMA's SrcC (even at
    NP + 3 wait states, which the pass-count rule accepts) and a load over an unread packed-f32
    source; an instruction reading the producer's result in between (the interlock) clears both."""
    hz = _hz()
    mf = "v_mfma_f32_16x16x4_f32 v[0:3], v4, v5, v[8:11]"
    late = [(1, mf), (2, "s_nop 10"), (3, "ds_read_b128 v[8:11], v6")]
    assert [h[0] for h in hz.scan_ldsrc(late)] == ["LDSRC"]
    assert not hz.scan_ldsrc([(1, mf), (2, "v_add_f32_e32 v7, v0, v7"), (3, "ds_read_b128 v[8:11], v6")])
    assert not hz.scan_ldsrc([(1, mf), (2, "s_nop 15"), (3, "s_nop 15"), (4, "ds_read_b128 v[8:11], v6")])
    pk = "v_pk_fma_f32 v[0:1], v[2:3], v[4:5], v[0:1]"
    assert [h[0] for h in hz.scan_pkwar([(1, pk), (2, "s_nop 7"), (3, "ds_read_b64 v[2:3], v6")])] == ["PKWAR"]
    assert not hz.scan_pkwar([(1, pk), (2, "v_mov_b32_e32 v7, v0"), (3, "ds_read_b64 v[2:3], v6")])
