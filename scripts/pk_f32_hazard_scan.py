#!/usr/bin/env python3
"""Find packed-FP32 VALU instructions (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 / v_pk_mov_b32)
that read a VGPR written by the IMMEDIATELY preceding VALU instruction (no s_nop or other
instruction between them), in every kernel of a .s file (or those whose symbol contains the
substring), split by the writer's kind (packed or 32-bit).

usage: pk_f32_hazard_scan.py FILE.s [SYMBOL_SUBSTRING] [-v]"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
PK = ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_mov_b32")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(4) is not None:
            out.add((m.group(1), int(m.group(4))))
        else:
            out.update((m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else None
    verbose = "-v" in sys.argv
    name, prev, hits = None, None, {}
    total = {"after_32bit_valu": 0, "after_pk_valu": 0}
    for raw in open(path):
        line = raw.rstrip("\n")
        m = re.match(r"^(_Z\S+|[A-Za-z_]\w*):", line)
        if m and not line.startswith("."):
            name, prev = m.group(1), None
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        if name is None or (want and want not in name):
            prev = None
            continue
        op = s.split()[0]
        ops = [o.strip() for o in s[len(op):].split(",")] if len(s) > len(op) else []
        if op.startswith(PK) and prev is not None:
            pop, pdst = prev
            srcs = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
            if pdst & srcs:
                kind = "after_pk_valu" if pop.startswith(PK) else "after_32bit_valu"
                total[kind] += 1
                hits.setdefault(name, []).append((kind, prev_line, s))
        if op.startswith("v_") and not op.startswith("v_mfma") and ops:
            prev, prev_line = (op, regs(ops[0])), s
        else:
            prev = None
    for n, hs in hits.items():
        k32 = sum(1 for h in hs if h[0] == "after_32bit_valu")
        print(f"{n[:100]}: {k32} after a 32-bit VALU writer, {len(hs) - k32} after a packed writer")
        if verbose:
            for h in hs:
                print("    ", h)
    print("total", total)


if __name__ == "__main__":
    main()
