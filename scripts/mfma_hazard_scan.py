#!/usr/bin/env python3
"""Scan one kernel's .s (hipcc -S) for the closest MFMA-related register dependencies, in program
order within straight-line code: per category, the minimum number of issue slots between the two
instructions (s_nop N counts N + 1). Used to compare two builds of one kernel (a passing and a
failing one) for a dependency the compiler may have spaced too tightly.

usage: mfma_hazard_scan.py FILE.s SYMBOL_SUBSTRING [--show CATEGORY]"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(4) is not None:
            out.add((m.group(1), int(m.group(4))))
        else:
            out.update((m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def kernel_lines(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) or (sym in l and l.endswith(":") is False and l.startswith("_Z") and sym in l.split(":")[0]))
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.split(";")[0].strip()
        if s:
            out.append(s)
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    show = sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--show" else None
    ins = []
    for s in kernel_lines(path, sym):
        if s.endswith(":"):
            ins.append(("LABEL", s, set(), set()))
            continue
        op = s.split()[0]
        ops = [o.strip() for o in s[len(op):].split(",")] if len(s) > len(op) else []
        ins.append((op, s, ops, None))
    best = {}
    examples = {}

    def note(cat, d, a, b):
        if cat not in best or d < best[cat]:
            best[cat] = d
            examples[cat] = (a, b)

    for i, (op, s, ops, _) in enumerate(ins):
        if op == "LABEL":
            continue
        is_mfma = op.startswith("v_mfma")
        is_valu = op.startswith("v_") and not is_mfma
        if not (is_mfma or is_valu):
            continue
        if is_mfma:
            dst, sa, sb, sc = regs(ops[0]), regs(ops[1]), regs(ops[2]), regs(ops[3])
        else:
            dst = regs(ops[0]) if ops else set()
        d = 0
        for j in range(i + 1, min(len(ins), i + 40)):
            op2, s2, ops2, _ = ins[j]
            if op2 == "LABEL":
                continue  # keep scanning through fallthrough labels
            if op2 in ("s_endpgm", "s_branch") or op2.startswith("s_cbranch"):
                break
            if op2 == "s_nop":
                d += int(s2.split()[1], 0) + 1
                continue
            is_m2 = op2.startswith("v_mfma")
            is_v2 = op2.startswith("v_") and not is_m2
            is_ds_w = op2.startswith(("ds_write", "ds_bpermute", "global_store", "buffer_store"))
            if is_m2:
                dst2, sa2, sb2, sc2 = regs(ops2[0]), regs(ops2[1]), regs(ops2[2]), regs(ops2[3])
                src2, wr2 = sa2 | sb2 | sc2, dst2
            elif is_v2:
                wr2 = regs(ops2[0]) if ops2 else set()
                src2 = set().union(*[regs(o) for o in ops2[1:]]) if len(ops2) > 1 else set()
            elif is_ds_w:
                wr2 = set()
                src2 = set().union(*[regs(o) for o in ops2]) if ops2 else set()
            else:
                wr2 = regs(ops2[0]) if (op2.startswith(("ds_read", "global_load", "buffer_load")) and ops2) else set()
                src2 = set().union(*[regs(o) for o in ops2[1:]]) if len(ops2) > 1 else set()
            if is_mfma:
                if is_v2 and wr2 & sc:
                    note("mfma_srcC_then_valu_write(WAR)", d, s, s2)
                if is_v2 and wr2 & (sa | sb):
                    note("mfma_srcAB_then_valu_write(WAR)", d, s, s2)
                if (is_v2 or is_ds_w) and src2 & dst:
                    note("mfma_dst_then_valu/ds_read_of_it(RAW)", d, s, s2)
                if is_v2 and wr2 & dst:
                    note("mfma_dst_then_valu_write(WAW)", d, s, s2)
                if is_m2 and (sa2 | sb2) & dst:
                    note("mfma_dst_then_mfma_srcAB(RAW)", d, s, s2)
                if is_m2 and sc2 & dst and sc2 != dst:
                    note("mfma_dst_then_mfma_srcC_partial_overlap", d, s, s2)
                if is_m2 and sc2 & dst and sc2 == dst:
                    note("mfma_dst_then_mfma_srcC_same(RAW)", d, s, s2)
                if is_m2 and wr2 & (sa | sb | sc):
                    note("mfma_src_then_mfma_dst_write(WAR)", d, s, s2)
                if not is_m2 and not is_v2 and wr2 & (sc | dst):
                    note("mfma_then_load_into_srcC/dst(WAR/WAW)", d, s, s2)
            else:
                if is_m2 and dst & (sa2 | sb2):
                    note("valu_write_then_mfma_srcAB(RAW)", d, s, s2)
                if is_m2 and dst & sc2:
                    note("valu_write_then_mfma_srcC(RAW)", d, s, s2)
            d += 1
    for k in sorted(best):
        print(f"{k:45s} min slots {best[k]:3d}   e.g. [{examples[k][0]}] -> [{examples[k][1]}]")


if __name__ == "__main__":
    main()
