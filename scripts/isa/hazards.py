#!/usr/bin/env python3
"""Static MFMA -> VALU hazard listing for one kernel's ISA (settle the
consumer-side env step's run-to-run differences statically).

For every MFMA, every later vector instruction within WINDOW issue slots that touches one of
its registers is listed with the number of wait states between them (each instruction = 1,
`s_nop N` = N + 1), by kind:
  RAW  VALU/VMEM/DS reads the MFMA's destination
  WAW  VALU/VMEM/DS writes the MFMA's destination
  WARc VALU writes the MFMA's SrcC (read over the MFMA's passes)
  WARab VALU writes SrcA/SrcB
  MRAW a later MFMA reads this MFMA's destination as SrcA/SrcB (SrcC chaining is exempt)
The scan follows the text order (fall-through), which is conservative at branch targets.
Pass counts (4 cycles each), measured on gfx950 (scripts/micro/mfma_mix.hip): 16x16x4 f32 8,
16x16x32 bf16 4, 16x16x16 bf16 4.  The requirement quoted beside each hit is the CDNA3/CDNA4
ISA rule for XDL ops, NumPasses + 2 wait states for RAW/WAW/MRAW and NumPasses for a SrcC
WAR (conservative reading); anything below it would be a missed hazard.
usage: hazards.py FILE.s SYMBOL_SUBSTRING [WINDOW]
build: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S [-DRD_CP_VARIANT] distill.hip"""
import re
import sys

PASSES = {"v_mfma_f32_16x16x4_f32": 8, "v_mfma_f32_16x16x4f32": 8, "v_mfma_f32_16x16x32_bf16": 4,
          "v_mfma_f32_16x16x16_bf16": 4, "v_mfma_f32_16x16x16bf16_1k": 4}


def regs(tok):
    """VGPR/AGPR numbers of one operand token ('v7', 'v[4:7]', 'a[0:3]') as a set of ('v', n)."""
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), k) for k in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"([va])(\d+)", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def operands(line):
    body = line.split(None, 1)
    if len(body) < 2:
        return []
    ops = [o.strip() for o in re.split(r",\s*(?![^\[]*\])", body[1].split(";")[0])]
    return [o.split()[0] if o else o for o in ops]


def scan(path, sym, window=24):
    """[(kind, wait states, requirement, MFMA line, MFMA op, line, instruction)] of one kernel."""
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    code = []
    for i in range(start, end + 1):
        l = lines[i].strip()
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        code.append((i + 1, l))
    hits = []
    for idx, (ln, l) in enumerate(code):
        op = l.split()[0]
        if not op.startswith("v_mfma"):
            continue
        o = operands(l)
        dst, a, b, c = (regs(x) for x in (o + ["", "", "", ""])[:4])
        npass = PASSES.get(op, 8)
        ws = 0
        for ln2, l2 in code[idx + 1: idx + 1 + window]:
            op2 = l2.split()[0]
            if op2 == "s_nop":
                ws += int(l2.split()[1], 0) + 1
                continue
            o2 = operands(l2)
            if op2.startswith("v_mfma"):
                d2, a2, b2, c2 = (regs(x) for x in (o2 + ["", "", "", ""])[:4])
                if (a2 | b2) & dst:
                    hits.append(("MRAW", ws, npass + 2, ln, op, ln2, l2))
                ws += 1
                continue
            if not (op2.startswith("v_") or op2.startswith("ds_") or op2.startswith(("global_", "buffer_"))):
                ws += 1
                continue
            w = regs(o2[0]) if o2 and not op2.startswith(("ds_write", "global_store", "buffer_store")) else set()
            r = set().union(*(regs(x) for x in (o2[1:] if w else o2))) if o2 else set()
            if r & dst:
                hits.append(("RAW", ws, npass + 2, ln, op, ln2, l2))
            if w & dst:
                hits.append(("WAW", ws, npass + 2, ln, op, ln2, l2))
            if w & (c - dst):
                hits.append(("WARc", ws, npass, ln, op, ln2, l2))
            if w & (a | b):
                hits.append(("WARab", ws, 1, ln, op, ln2, l2))
            ws += 1
    return hits, code


def main():
    path, sym = sys.argv[1], sys.argv[2]
    window = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    hits, code = scan(path, sym, window)
    short = [h for h in hits if h[1] < h[2]]
    kinds = {}
    for h in hits:
        kinds.setdefault((h[0], h[4]), []).append(h[1])
    print(f"{sym}: {sum(1 for _, l in code if l.startswith('v_mfma'))} MFMAs, {len(hits)} register-sharing "
          f"instructions within {window} slots")
    for (k, op), ws in sorted(kinds.items()):
        print(f"  {k:5s} after {op:28s} n={len(ws):4d} min wait states {min(ws):3d}")
    print(f"below the conservative requirement: {len(short)}")
    for h in short[:40]:
        print(f"  {h[0]:5s} ws {h[1]:2d} < {h[2]:2d}: line {h[3]} {h[4]} -> line {h[5]}: {h[6][:90]}")


if __name__ == "__main__":
    main()
