#!/usr/bin/env python3
"""ISA audit of the built kernel library (the gfx950 code objects inside liblsa_kernels.so).

A read of a VGPR in the issue slot right after the instruction that writes it can return the OLD
value on MI355X for some writer / reader pairs unless a wait state separates them. hipcc's hazard
recognizer inserts those wait states; this audit checks the binary that ships instead of trusting
it. The rules and their evidence (scripts/probes/pk_hazard_gen.py: every writer / gap / reader
combination as raw inline asm, compared bitwise against the same sequence with 16 wait states, at
one wave per SIMD, eight waves per SIMD and four hazard waves beside four MFMA-issuing waves per
SIMD, 8.4-67 M lane tests per case; profiles/r6_isa_hazards.md):

* R1 ``trans``: a transcendental VALU op (v_exp / v_log / v_rcp / v_rsq / v_sqrt / v_sin / v_cos)
  whose result is read by the NEXT VALU instruction - packed, DPP or plain 32-bit: 22 % of lanes
  read the stale value. MEASURED HAZARD.
* R2 ``dpp``: any VALU write of a VGPR that the NEXT instruction reads through DPP: 44-49 % stale.
  MEASURED HAZARD.
* R3 ``valu32->pk``: a 32-bit VALU write of a VGPR that the next packed-FP32 instruction
  (v_pk_fma / mul / add_f32, v_pk_mov_b32) reads. NOT reproduced on hardware: 0 stale reads in
  every case, including the exact round-5 GEMV site (two v_fma_f32 updating both halves of a pair,
  then v_pk_fma_f32 accumulating into it) beside MFMA-issuing waves. Kept as a conservative rule:
  the product build (-fno-slp-vectorize, csrc/build.py) forms no packed FP32 from scalar code, so
  it costs nothing, and an SLP-vectorised build of the round-5 shared GEMV body computed wrong rows
  for a reason this rule's pattern does not explain (profiles/r5_gemv_nondeterminism.md, round-6
  section).

One slot is the whole window: with one wait state (s_nop 0) or one independent VALU instruction
between writer and reader, every case of every rule read the new value; distance-2 writers never
need a wait state. The shipped library has 0 findings under all three rules (the packed-FP32
instructions that remain come from explicit vector code, each behind a packed writer or at a
distance).

usage: python csrc/isa_audit.py [path/to/liblsa_kernels.so] [arch]   (exit 1 on any finding)"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LLVM = os.path.join(ROCM, "lib", "llvm", "bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--{arch}"
PK = ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_mov_b32")
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")
REG = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")
RULES = ("trans", "dpp", "valu32->pk")


def _vregs(tok: str) -> set:
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(so_path: str, arch: str = "gfx950") -> list:
    """Disassembly text of every ``arch`` code object bundled in the library's .hip_fatbin."""
    texts = []
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", so_path,
                        os.path.join(td, "discard.so")], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, st in enumerate(starts):
            chunk = data[st:starts[i + 1] if i + 1 < len(starts) else len(data)]
            cp, co = os.path.join(td, f"b{i}.bin"), os.path.join(td, f"b{i}.co")
            with open(cp, "wb") as f:
                f.write(chunk)
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", f"--input={cp}",
                                f"--targets={TARGET.format(arch=arch)}", f"--output={co}", "--unbundle"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            d = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                               text=True)
            texts.append(d.stdout)
    return texts


def _is_dpp(op: str, text: str) -> bool:
    return "_dpp" in op or any(k in text for k in (" quad_perm:", " row_shl:", " row_shr:", " row_ror:",
                                                     " row_mirror", " row_half_mirror", " row_bcast",
                                                     " row_share:", " row_xmask:", " wave_"))


def audit_text(text: str, rules=RULES) -> tuple:
    """(findings, packed_fp32_count): findings = [(rule, kernel, writer, reader)] for every
    reader in the issue slot right after a writer of one of its source VGPRs."""
    findings, n_pk = [], 0
    kernel, prev = None, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line.strip())
        if m:
            kernel, prev = m.group(1), None
            continue
        s = line.split("//")[0].strip()
        if not s:
            continue
        op = s.split()[0]
        ops = [o.strip() for o in s[len(op):].split(",")] if len(s) > len(op) else []
        is_valu = op.startswith("v_") and not op.startswith(("v_mfma", "v_smfma"))
        if op.startswith(PK):
            n_pk += 1
        if is_valu and prev is not None:
            srcs = set().union(*[_vregs(o) for o in ops[1:]]) if len(ops) > 1 else set()
            if prev[2] & srcs:
                pop = prev[0]
                if "trans" in rules and pop.startswith(TRANS):
                    findings.append(("trans", kernel, prev[1], s))
                # DPP reads its first source through the permute network
                if "dpp" in rules and _is_dpp(op, s) and len(ops) > 1 and prev[2] & _vregs(ops[1]):
                    findings.append(("dpp", kernel, prev[1], s))
                if "valu32->pk" in rules and op.startswith(PK) and not pop.startswith(PK):
                    findings.append(("valu32->pk", kernel, prev[1], s))
        if is_valu and ops:
            prev = (op, s, _vregs(ops[0]))
        else:
            prev = None
    return findings, n_pk


def audit(so_path: str, arch: str = "gfx950") -> dict:
    findings, n_pk, n_obj = [], 0, 0
    for t in disassemble(so_path, arch):
        f, n = audit_text(t)
        findings += f
        n_pk += n
        n_obj += 1
    by_rule = {r: sum(1 for f in findings if f[0] == r) for r in RULES}
    return {"code_objects": n_obj, "packed_fp32_instructions": n_pk, "findings": findings, "by_rule": by_rule}


def main() -> None:
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                              "llm_sharding_amd", "_native", "liblsa_kernels.so")
    arch = sys.argv[2] if len(sys.argv) > 2 else "gfx950"
    res = audit(so, arch)
    for r, k, w, rd in res["findings"][:20]:
        print(f"{r:10s} {k[:80]}: [{w}] -> [{rd}]")
    print(f"code objects {res['code_objects']}, packed FP32 instructions {res['packed_fp32_instructions']}, "
          f"back-to-back findings by rule {res['by_rule']}")
    sys.exit(1 if res["findings"] or not res["code_objects"] else 0)


if __name__ == "__main__":
    main()
