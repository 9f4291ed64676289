#!/usr/bin/env python3
"""ISA audit of the built kernel library (gfx950 code objects inside liblsa_kernels.so).

Checks the one hazard pattern found to corrupt results on MI355X with ROCm 7.2's compiler
(profiles/r5_gemv_nondeterminism.md): a packed-FP32 VALU instruction (v_pk_fma_f32 /
v_pk_mul_f32 / v_pk_add_f32 / v_pk_mov_b32) issued IMMEDIATELY after a VALU instruction that
writes one of its source VGPRs, with no wait state between them. hipcc inserts the wait state
(an s_nop) when the writer is itself a packed instruction but not when it is a 32-bit one; the
decode GEMV built that way computed wrong rows nondeterministically. The library is built with
-fno-slp-vectorize (csrc/build.py), which keeps the compiler from forming packed FP32 math at
all; this audit proves it on the binary that ships.

usage: python csrc/isa_audit.py [path/to/liblsa_kernels.so]   (exit 1 on any finding)"""
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
REG = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")


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
                                f"--targets={TARGET.format(arch=arch)}", f"--output={co}", "--unbundle"], capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            d = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                               text=True)
            texts.append(d.stdout)
    return texts


def audit_text(text: str) -> tuple:
    """(findings, packed_fp32_count): findings = [(kernel, writer, reader)]."""
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
        if op.startswith(PK):
            n_pk += 1
            if prev is not None:
                srcs = set().union(*[_vregs(o) for o in ops[1:]]) if len(ops) > 1 else set()
                if prev[1] & srcs:
                    findings.append((kernel, prev[0], s))
        if op.startswith("v_") and not op.startswith(("v_mfma", "v_smfma")) and ops:
            prev = (s, _vregs(ops[0]))
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
    return {"code_objects": n_obj, "packed_fp32_instructions": n_pk, "findings": findings}


def main() -> None:
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                              "llm_sharding_amd", "_native", "liblsa_kernels.so")
    res = audit(so)
    for k, w, r in res["findings"][:20]:
        print(f"{k[:90]}: [{w}] -> [{r}]")
    print(f"code objects {res['code_objects']}, packed FP32 instructions {res['packed_fp32_instructions']}, "
          f"VALU -> packed-FP32 back-to-back dependencies {len(res['findings'])}")
    sys.exit(1 if res["findings"] else 0)


if __name__ == "__main__":
    main()
