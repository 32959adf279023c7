#!/usr/bin/env python3
"""rebuild the ISA of the r03w/r03x library (b098fce's distill.hip with
972b9ac's inline-asm non-temporal partial row put back) and of b098fce itself, from git history
only (nothing runs on a GPU), and scan both with scripts/isa/hazards.py.

usage: python scripts/isa/r03x_rebuild.py OUTDIR   (record: profiles/r04_r03x_isa.txt)"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts", "isa"))
import hazards as hz  # noqa: E402

HIPCC = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
         "-Wno-unused-command-line-argument", "--cuda-device-only", "-S"]


def show(rev, path):
    return subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{path}"], check=True, capture_output=True,
                          text=True).stdout


def asm_row(src):
    """b098fce's distill.hip with the rollout's partial row as 972b9ac wrote it (inline asm nt)."""
    src = src.replace("#include <new>\n", "#include <new>\n#include <type_traits>\n", 1)
    src = src.replace("""    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
""", """    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
constexpr unsigned WS_NT_MIN_GRID = 128;
__device__ __forceinline__ void st4_nt(float* p, f32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
}
""", 1)
    old = """            gst<kWsNt>(reinterpret_cast<f32x4*>(a.ws + ws_index(4 * p4, blockIdx.x, gridDim.x)),
                       (ld4(lds + q) + ld4(lds + RPAD + q)) + (ld4(lds + 2 * RPAD + q) + ld4(lds + 3 * RPAD + q)));"""
    new = """            float* w = a.ws + ws_index(4 * p4, blockIdx.x, gridDim.x);
            const f32x4 v = (ld4(lds + q) + ld4(lds + RPAD + q)) + (ld4(lds + 2 * RPAD + q) + ld4(lds + 3 * RPAD + q));
            if constexpr (decltype(nt)::value) st4_nt(w, v);
            else st4(w, v);"""
    assert src.count(old) == 1
    src = src.replace(old, new)
    loop = src[src.index("#pragma unroll\n    for (int u = 0; u < (P_PAD / 4 + BLOCK - 1) / BLOCK; ++u) {"):]
    loop = loop[:loop.index("    STAMP(7);")]
    body = loop.replace("\n", "\n    ")
    src = src.replace(loop, "auto store_row = [&](auto nt) {\n" + body.rstrip() + "\n    };\n"
                      "    if (WS_NT_MIN_GRID == 0 || gridDim.x >= WS_NT_MIN_GRID) store_row(std::true_type{});\n"
                      "    else store_row(std::false_type{});\n", 1)
    return src


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/r03x"
    csrc = os.path.join(out, "src", "csrc")
    os.makedirs(csrc, exist_ok=True)
    os.makedirs(os.path.join(out, "include"), exist_ok=True)
    for h in ("rd_common.h", "rd_physics.h", "rd_comm_impl.h"):
        open(os.path.join(csrc, h), "w").write(show("b098fce", f"reacherdistilation_amd/csrc/{h}"))
    for h in subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", "b098fce", "include/"], check=True,
                            capture_output=True, text=True).stdout.split():
        open(os.path.join(out, h), "w").write(show("b098fce", h))
    base = show("b098fce", "reacherdistilation_amd/csrc/distill.hip")
    isa = {}
    for tag, src in (("b098fce", base), ("r03w", asm_row(base))):
        p = os.path.join(csrc, f"distill_{tag}.hip")
        open(p, "w").write(src)
        isa[tag] = os.path.join(out, f"{tag}.s")
        subprocess.run(HIPCC + ["-o", isa[tag], p], check=True, capture_output=True)
    for tag, path in isa.items():
        for name, code in hz.functions(path).items():
            if "rollout_kernel" not in name:
                continue
            hits = hz.scan_code(code, 40)
            per = collections.Counter(h[0] for h in hits)
            low = collections.Counter(h[0] for h in hz.violations(hits))
            stores = [l for _, l in code if re.match(r"global_store_dwordx4 .* nt$", l)]
            mins = {k: min(h[1] for h in hits if h[0] == k) for k in per}
            print(f"{tag:8s} {name[32:60]} asm-nt stores {len(stores)} below requirement {dict(low) or 0}")
            print("         min wait states per class:", dict(sorted(mins.items())))


if __name__ == "__main__":
    main()
