#!/usr/bin/env python3
"""Static check of hipcc's vmcnt waits in one kernel's .s: explore every control-flow path (loops
included, until the (block, in-flight loads) state repeats) and report any instruction that reads a
VGPR / AGPR whose vector-memory load may still be in flight (not yet covered by an s_waitcnt
vmcnt(N) that retires it). Loads, stores and LDS-DMA count together in vmcnt, in issue order.

LGKM=1 in the environment checks the LDS / scalar-memory counter instead (ds_read*, ds_bpermute,
ds_*_rtn, s_load*, s_buffer_load*; a scalar load in flight makes only lgkmcnt(0) a safe wait, so
any wait above 0 retires none of the scalar loads).

usage: vmcnt_check.py FILE.s [kernel-symbol-substring]"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(tok: str):
    out = set()
    for m in REG.finditer(tok):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            out.update((k, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(lines):
    insts, labels = [], {}
    for no, raw in lines:
        s = raw.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.endswith(":") and s.startswith(".LBB"):
                labels[s[:-1]] = len(insts)
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(insts)
            continue
        insts.append((no, s))
    return insts, labels


LGKM = __import__("os").environ.get("LGKM") == "1"


def classify(s: str):
    op = s.split()[0]
    if LGKM:
        rest = s[len(op):].strip()
        ops = [o.strip() for o in rest.split(",")] if rest else []
        ev = op.startswith(("ds_read", "ds_bpermute", "ds_permute", "s_load", "s_buffer_load")) or (
            op.startswith("ds_") and "_rtn" in op)
        dst, srcs = set(), set()
        if ev:
            dst = regs(ops[0]) if ops else set()
            if op.startswith("s_"):
                dst = {("s", 0)}  # marker: scalar load in flight
            for o in ops[1:]:
                srcs |= regs(o)
        elif op.startswith("s_"):
            pass
        else:
            if ops and not op.startswith(("ds_write", "global_store", "buffer_store")):
                dst = regs(ops[0])
                for o in ops[1:]:
                    srcs |= regs(o)
            else:
                for o in ops:
                    srcs |= regs(o)
        return op, ev, dst, srcs
    rest = s[len(op):].strip()
    ops = [o.strip() for o in rest.split(",")] if rest else []
    is_vm = op.startswith(("global_", "buffer_", "flat_", "scratch_")) and "wbl2" not in op and "inv" not in op
    is_load = is_vm and ("load" in op or "atomic" in op and "glc" in s or op.endswith("_lds"))
    lds_dma = is_vm and (" lds" in s or op.startswith("global_load_lds"))
    dst, srcs = set(), set()
    if is_vm and is_load and not lds_dma:
        dst = regs(ops[0]) if ops else set()
        for o in ops[1:]:
            srcs |= regs(o)
    elif op.startswith(("global_store", "buffer_store", "ds_write", "flat_store", "scratch_store")) or lds_dma:
        for o in ops:
            srcs |= regs(o)
    elif op.startswith(("s_", )):
        pass
    else:
        if ops:
            dst = regs(ops[0])
        for o in ops[1:]:
            srcs |= regs(o)
    return op, is_vm, dst, srcs


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    lines = list(enumerate(open(path).read().splitlines(), 1))
    # kernel bodies: from "<sym>:" to s_endpgm
    bodies, cur, name = [], None, None
    for no, raw in lines:
        m = re.match(r"^([A-Za-z_][\w$.]*):\s*(;.*)?$", raw)
        if m and not raw.startswith(".") and cur is None and "LBB" not in m.group(1):
            name, cur = m.group(1), []
            continue
        if cur is not None:
            cur.append((no, raw))
            if raw.strip().startswith("s_endpgm") and not any(r.strip().startswith(".LBB") for _, r in lines[no:no + 3]):
                pass
            if raw.strip().startswith(".Lfunc_end"):
                bodies.append((name, cur))
                cur = None
    bad_total = 0
    for name, body in bodies:
        if want and want not in name:
            continue
        insts, labels = parse(body)
        info = [classify(s) for _, s in insts]
        seen = set()
        stack = [(0, ())]
        bad = {}
        steps = 0
        while stack:
            pc, pend = stack.pop()
            while pc < len(insts):
                key = (pc, pend)
                if key in seen:
                    break
                seen.add(key)
                steps += 1
                if steps > 2_000_000:
                    print(name, "state space too large; stopped")
                    stack = []
                    break
                no, s = insts[pc]
                op, is_vm, dst, srcs = info[pc]
                m = re.search(r"lgkmcnt\((\d+)\)" if LGKM else r"vmcnt\((\d+)\)", s)
                if op == "s_waitcnt" and m:
                    n = int(m.group(1))
                    if LGKM and n > 0 and any(("s", 0) in d for _, d in pend):
                        pass  # scalar loads return out of order: only lgkmcnt(0) retires them
                    else:
                        pend = pend[len(pend) - n:] if n < len(pend) else pend
                    if n == 0:
                        pend = ()
                pending_regs = {}
                for i, (lno, d) in enumerate(pend):
                    for r in d:
                        pending_regs[r] = lno
                hit = (srcs | (dst if not is_vm else set())) & set(pending_regs)
                if hit:
                    r = sorted(hit)[0]
                    bad.setdefault(no, (s, pending_regs[r], r))
                if is_vm:
                    pend = pend + ((no, frozenset(dst)),)
                if op == "s_endpgm":
                    break
                if op == "s_branch":
                    pc = labels[s.split()[1]]
                    continue
                if op.startswith("s_cbranch"):
                    tgt = s.split()[1]
                    stack.append((labels[tgt], pend))
                pc += 1
        for no, (s, lno, r) in sorted(bad.items()):
            print(f"{name[:60]}: line {no}: '{s}' reads {r[0]}{r[1]} loaded at line {lno} (maybe in flight)")
        bad_total += len(bad)
        print(f"{name[:80]}: {len(bad)} hazard(s), {steps} states")
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
