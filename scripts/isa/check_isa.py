#!/usr/bin/env python3
"""Every hazard class the hygiene tests assert, on one ISA file (a variant build's distill.hip):
LDSRC by interlock, PKWAR, packed-f32 ops in the rollout instances, the generic scan.
  check_isa.py ISA.s"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import hazards as hz  # noqa: E402


def main():
    path = sys.argv[1]
    fns = hz.functions(path)
    bad = {}
    for name, code in fns.items():
        for kind, hits in (("LDSRC", hz.scan_ldsrc(code)), ("PKWAR", hz.scan_pkwar(code)),
                           ("SCAN", hz.violations(hz.scan_code(code, 40)))):
            if hits:
                bad.setdefault(name[-60:], []).append((kind, [h[:6] for h in hits[:2]]))
        if "rollout_kernel" in name:
            pk = [l for _, l in code if l.startswith(hz.PK_F32)]
            if pk:
                bad.setdefault(name[-60:], []).append(("PK_F32", pk[:2]))
    print(f"{len(fns)} functions, {len(bad)} with hazards")
    for k, v in bad.items():
        print(k, v)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
