#!/usr/bin/env python3
"""VALU instructions of one rollout_kernel instance by ROLE, weighted by how often each runs
("split the VALU count by role and phase").

Reads an ISA file compiled with line tables (hipcc -O3 -g ... --cuda-device-only -S): every
instruction is attributed to the source function its `.loc` line falls in (distill.hip's
helpers and kernel sections, rd_physics.h's functions), and every basic block gets an execution
weight from the control flow: natural loops are found from the back-edges, and a block runs
`trips ** depth` times per wave for the loop depth it sits at (trips given per depth, e.g. 4 groups
per pair and 4 tiles per group at c4).  Static attribution, so the weights are the kernel's
loop structure, not a measurement: the PMC pass (SQ_INSTS_VALU) gives the measured total to
compare with.

usage: valu_roles.py ISA.s SYMBOL_SUBSTRING DEPTH_TRIPS(e.g. 4,4) [SOURCE.hip]"""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import hazards as hz  # noqa: E402

SRC_DEFAULT = "reacherdistilation_amd/csrc/distill.hip"


def function_ranges(src):
    """[(start_line, name)] of the device functions / lambdas / kernel sections of a source."""
    out = []
    pat = re.compile(r"^\s*(?:template\s*<[^>]*>\s*)?(?:__device__|__global__)[^(]*?\b(\w+)\s*\(")
    for i, l in enumerate(open(src).read().split("\n"), 1):
        m = pat.match(l)
        if m:
            out.append((i, m.group(1)))
        for tag in ("auto bwd_tile", "auto end_group", "auto group_obs", "// ---------------------------------------------------------- env.step",
                    "// ============================================================ producer wave",
                    "// ============================================================ consumer wave",
                    "// loss", "// dW3 partials", "// hand the tile over", "// ------------------------------------------------------------ this wave's share",
                    "// dH1 = W2 . dZ2", "// dW1 (+ db1", "// db2 partials and dW2", "// read the whole slot"):
            if tag in l:
                out.append((i, tag.strip("/ =-").split("(")[0].strip()))
    return sorted(out)


def role_of(ranges, line):
    name = "?"
    for start, n in ranges:
        if start <= line:
            name = n
        else:
            break
    return name


def main():
    path, sym, trips = sys.argv[1], sys.argv[2], [int(x) for x in sys.argv[3].split(",")]
    src = sys.argv[4] if len(sys.argv) > 4 else SRC_DEFAULT
    lines = open(path).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = m.group(3)
    # the function's lines with their .loc
    name = next(n for n in hz.functions(path) if sym in n)
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    code, loc = [], (0, 0)
    for i in range(start + 1, len(lines)):
        l = lines[i].split(";")[0].strip()
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (int(m.group(1)), int(m.group(2)))
            continue
        if not l or (l.startswith(".") and not l.endswith(":")):
            continue
        code.append((i + 1, l, loc))
    insts, succ = hz._cfg([(ln, l) for ln, l, _ in code])
    locs = [lc for _, l, lc in code if not l.endswith(":")]
    # loop depth per instruction: natural loops of the back-edges (target index <= source index)
    n = len(insts)
    pred = collections.defaultdict(list)
    for k, ss in enumerate(succ):
        for s2 in ss:
            pred[s2].append(k)
    depth = [0] * n
    for k, ss in enumerate(succ):
        for h in ss:
            if h <= k:   # back-edge k -> h: the loop is every instruction reaching k without passing h
                body, stack = {h}, [k]
                while stack:
                    x = stack.pop()
                    if x in body:
                        continue
                    body.add(x)
                    stack.extend(p for p in pred[x] if p not in body)
                for x in body:
                    depth[x] += 1
    ranges = function_ranges(src)
    hranges = {}
    per_role = collections.Counter()
    per_role_static = collections.Counter()
    mfma_w = 0.0
    for k, ((ln, l), (f, line)) in enumerate(zip(insts, locs)):
        op = l.split()[0]
        d = min(depth[k], len(trips))
        w = 1.0
        for t in trips[:d]:
            w *= t
        if op.startswith(("v_mfma", "v_smfmac")):
            mfma_w += w
            continue
        if not op.startswith("v_"):
            continue
        fn = files.get(f, "?")
        if fn.endswith(src.rsplit("/", 1)[-1]):
            role = role_of(ranges, line)
        else:
            if fn not in hranges:
                import os
                h = "reacherdistilation_amd/csrc/" + fn
                hranges[fn] = function_ranges(h) if os.path.exists(h) else []
            role = fn.rsplit(".", 1)[0] + ":" + role_of(hranges[fn], line)
        if op.startswith(hz.TRANS):
            role += " [trans]"
        per_role[role] += w
        per_role_static[role] += 1
    tot = sum(per_role.values())
    print(f"{sym}: weighted VALU {tot:.0f} per wave pass (trips per loop depth {trips}), weighted MFMA {mfma_w:.0f}, "
          f"VALU/MFMA {tot / max(mfma_w, 1):.2f}")
    for r, v in per_role.most_common():
        print(f"  {v:9.0f}  {100 * v / tot:5.1f} %  static {per_role_static[r]:5d}  {r}")


if __name__ == "__main__":
    main()
