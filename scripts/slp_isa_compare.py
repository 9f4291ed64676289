#!/usr/bin/env python3
"""Per-kernel FP32 instruction mix of two builds of the kernel library (product: no SLP; probe:
SLP on), restricted to the kernels whose names match a pattern - the ISA side of
scripts/slp_kernel_diff.py (which names the kernels that compute different bits).

For each kernel: counts of packed FP32 (v_pk_fma/mul/add_f32), scalar FMA (v_fma_f32 / v_fmac_f32),
v_mul_f32, v_add_f32 and trans ops. A build that forms v_pk_mul_f32 + v_pk_add_f32 where the other
forms v_fma_f32 (or the reverse) rounds once instead of twice per multiply-add: different bits,
deterministically - FMA contraction, not a hazard.

usage: python scripts/slp_isa_compare.py [pattern ...]   (default: attention kernels)"""
from __future__ import annotations

import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "csrc"))
from isa_audit import disassemble  # noqa: E402

GROUPS = {
    "pk_fma": ("v_pk_fma_f32",), "pk_mul": ("v_pk_mul_f32",), "pk_add": ("v_pk_add_f32",),
    "fma": ("v_fma_f32", "v_fmac_f32"), "mul": ("v_mul_f32",), "add": ("v_add_f32",),
    "trans": ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32"),
}


def mix(so: str) -> dict:
    out = collections.defaultdict(collections.Counter)
    for text in disassemble(so):
        kernel = None
        for line in text.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line.strip())
            if m:
                kernel = m.group(1)
                continue
            s = line.split("//")[0].strip()
            if not s or kernel is None:
                continue
            op = s.split()[0]
            base = re.sub(r"_e(32|64)(_dpp)?$", "", op)
            for g, names in GROUPS.items():
                if base in names:
                    out[kernel][g] += 1
    return out


def main() -> None:
    pats = sys.argv[1:] or ["attn"]
    a = mix(os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_kernels.so"))
    b = mix(os.path.join(ROOT, "probe_bin", "liblsa_kernels_slp.so"))
    keys = sorted(k for k in set(a) | set(b) if any(p in k for p in pats))
    print(f"{'kernel':70s} " + " ".join(f"{g:>13s}" for g in GROUPS))
    for k in keys:
        row = " ".join(f"{a[k][g]:>6d}/{b[k][g]:<6d}" for g in GROUPS)
        print(f"{k[:70]:70s} {row}")
    print("(each cell: product build / SLP build)")


if __name__ == "__main__":
    main()
