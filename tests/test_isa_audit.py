"""The shipped kernel library contains no VALU -> packed-FP32 back-to-back dependency (the
compiler pattern that made the decode GEMV compute wrong rows nondeterministically,
profiles/r5_gemv_nondeterminism.md): csrc/isa_audit.py disassembles the gfx950 code objects
inside liblsa_kernels.so. CPU-only (the disassembler runs here)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_kernels.so")


@pytest.mark.skipif(not os.path.exists(SO), reason="kernel library not built (python csrc/build.py)")
def test_library_has_no_valu_to_packed_fp32_hazard():
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    from isa_audit import audit
    res = audit(SO)
    assert res["code_objects"] >= 9, res
    assert not res["findings"], res["findings"][:10]


def test_audit_flags_the_pattern():
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    from isa_audit import audit_text
    bad = """0000000000001000 <k>:
\tv_fma_f32 v6, v38, v38, v6 // 000000001000: D5CB0006
\tv_fma_f32 v7, v39, v39, v7 // 000000001008: D5CB0007
\tv_pk_fma_f32 v[198:199], v[40:41], v[40:41], v[6:7] // 000000001010: D3B000C6
"""
    ok = bad.replace("\tv_pk_fma_f32", "\ts_nop 0\n\tv_pk_fma_f32")
    assert len(audit_text(bad)[0]) == 1 and audit_text(ok)[0] == []
