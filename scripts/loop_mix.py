#!/usr/bin/env python3
"""Instruction mix of every innermost loop of one kernel in a hipcc .s file (blocks LLVM tags with
'in Loop: Header=<header>'), per loop iteration: MFMA, LDS, DMA / VMEM, VALU, SALU, branches,
waits, barriers. usage: loop_mix.py FILE.s SYMBOL_SUBSTRING"""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    loops = collections.defaultdict(list)
    cur = None
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):(.*)$", l)
        if m or l.startswith("; %bb"):
            tag = l + (body[i + 1] if i + 1 < len(body) else "")
            h = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", tag)
            self_hdr = re.search(r"=>\s*This (Inner )?Loop Header: Depth=(\d+)", tag)
            if self_hdr and m:
                cur = (m.group(1)[1:], int(self_hdr.group(2)))
            elif h:
                cur = (h.group(1), int(h.group(2)))
            else:
                cur = None
            continue
        if cur:
            s = l.split(";")[0].strip()
            if s and not s.endswith(":"):
                loops[cur].append(s)
    for (hdr, depth), seg in loops.items():
        cnt = collections.Counter()
        for s in seg:
            op = s.split()[0]
            k = ("mfma" if op.startswith("v_mfma") else "waitcnt" if op.startswith("s_waitcnt") else
                 "barrier" if op.startswith("s_barrier") else "branch" if "branch" in op else
                 "nop" if op == "s_nop" else "salu" if op.startswith("s_") else
                 "ds_read" if op.startswith("ds_read") else "ds_other" if op.startswith("ds_") else
                 "vmem" if op.startswith(("global_", "buffer_")) else "valu" if op.startswith("v_") else op)
            cnt[k] += 1
        print(f"loop {hdr} depth {depth}: {len(seg)} insts {dict(cnt)}")


if __name__ == "__main__":
    main()
