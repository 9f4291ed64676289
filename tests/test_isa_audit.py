"""csrc/isa_audit.py: the shipped kernel library has no back-to-back hazard under any of the
audit's rules, each rule flags its pattern (and not the same pattern one wait state apart), and
the rules agree with the hardware: on the hazard probe's own ISA (scripts/probes/pk_hazard_gen.py)
the trans and DPP rules flag exactly the cases that read stale values on an MI355X
(profiles/r6_pk_hazard_probe.txt); and the bit_cast-of-a-vector-element miscompile behind the
round-5 "fdot2" report is reproduced and kept out of the product kernels. CPU-only (the
disassembler runs here)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "llm_sharding_amd", "_native", "liblsa_kernels.so")
sys.path.insert(0, os.path.join(ROOT, "csrc"))


def _audit_text(text):
    from isa_audit import audit_text
    return [f[0] for f in audit_text(text)[0]]


@pytest.mark.skipif(not os.path.exists(SO), reason="kernel library not built (python csrc/build.py)")
def test_library_has_no_back_to_back_hazard():
    from isa_audit import audit
    res = audit(SO)
    assert res["code_objects"] >= 9, res
    assert not res["findings"], res["findings"][:10]


K = "0000000000001000 <k>:\n"


def test_rule_valu32_to_packed():
    bad = K + """\tv_fma_f32 v6, v38, v38, v6 // 000000001000: D5CB0006
\tv_fma_f32 v7, v39, v39, v7 // 000000001008: D5CB0007
\tv_pk_fma_f32 v[198:199], v[40:41], v[40:41], v[6:7] // 000000001010: D3B000C6
"""
    assert _audit_text(bad) == ["valu32->pk"]
    assert _audit_text(bad.replace("\tv_pk_fma_f32", "\ts_nop 0\n\tv_pk_fma_f32")) == []
    # a packed writer in front of a packed reader is not this rule
    assert _audit_text(K + "\tv_pk_add_f32 v[6:7], v[6:7], v[8:9]\n\tv_pk_fma_f32 v[10:11], v[6:7], v[6:7], v[2:3]\n") == []


def test_rule_trans():
    bad = K + "\tv_exp_f32_e32 v40, v12\n\tv_add_f32_e32 v44, v40, v42\n"
    assert _audit_text(bad) == ["trans"]
    assert _audit_text(K + "\tv_rsq_f32_e32 v40, v12\n\tv_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n") == \
        ["trans", "valu32->pk"]
    # one independent VALU between writer and reader: the new value is read (measured)
    assert _audit_text(K + "\tv_exp_f32_e32 v40, v12\n\tv_mov_b32_e32 v48, v49\n\tv_add_f32_e32 v44, v40, v42\n") == []


def test_rule_dpp():
    bad = K + ("\tv_add_f32_e32 v40, v40, v12\n"
               "\tv_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n")
    assert _audit_text(bad) == ["dpp"]
    assert _audit_text(bad.replace("\tv_mov_b32_dpp", "\ts_nop 0\n\tv_mov_b32_dpp")) == []
    # the DPP instruction's other operands are read normally
    assert _audit_text(K + "\tv_add_f32_e32 v41, v40, v12\n"
                       "\tv_add_f32_dpp v44, v40, v41 row_shr:1 row_mask:0xf bank_mask:0xf\n") == []


def _measured_hazards():
    """{case name: stale reads anywhere} from the committed hardware run of the probe."""
    out = {}
    for line in open(os.path.join(ROOT, "profiles", "r6_pk_hazard_probe.txt")):
        m = re.match(r"^(\S+ \S+ \S+)\s+1w/SIMD (\d+)/\d+\s+8w/SIMD (\d+)/\d+\s+4w\+4mfma/SIMD (\d+)/\d+", line)
        if m:
            out[m.group(1)] = any(int(m.group(i)) for i in (2, 3, 4))
    return out


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_rules_match_the_hardware(tmp_path):
    """Rebuild the probe from its generator, audit its ISA, and map every finding back to its case:
    the trans and DPP rules flag exactly the cases measured stale on the MI355X; the conservative
    valu32->pk rule flags only cases measured CLEAN (it is not a hardware hazard)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts", "probes"))
    import pk_hazard_gen as gen
    cases = gen.gen()
    exe = str(tmp_path / "pk_hazard_probe")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "--offload-arch=gfx950", gen.SRC, "-o", exe], check=True,
                   capture_output=True)
    from isa_audit import audit_text, disassemble
    texts = disassemble(exe)
    assert texts
    flagged = {}
    for rule, kernel, _w, _r in audit_text(texts[0])[0]:
        ci = int(re.search(r"case_(\d+)", kernel).group(1))
        flagged.setdefault(" ".join(cases[ci]), set()).add(rule)
    measured = _measured_hazards()
    assert len(measured) == len(cases)
    stale = {c for c, v in measured.items() if v}
    by_hw_rules = {c for c, r in flagged.items() if r & {"trans", "dpp"}}
    assert by_hw_rules == stale, (sorted(stale - by_hw_rules), sorted(by_hw_rules - stale))
    pk_only = {c for c, r in flagged.items() if r == {"valu32->pk"}}
    assert pk_only and not (pk_only & stale)


def test_product_kernels_avoid_the_bit_cast_element_miscompile():
    """ROCm 7.2's hipcc reads element 0 for ``__builtin_bit_cast(T, v[k])`` when ``v`` is an
    ext_vector and ``k`` a (constant) index: four fdot2 calls on the four dwords of a 16-byte
    operand all read dword 0 (scripts/probes/fdot2_repro.hip, profiles/r6_fdot2_miscompile.md; the
    round-5 persistent-chain probe hit it). Product kernels never bit_cast a single-subscript
    element (copy it to a scalar first); the double-subscript uses (arrays OF vectors, e.g.
    acc[i][j]) are whole objects and compile correctly."""
    import glob
    pat = re.compile(r"__builtin_bit_cast\(\s*[\w:]+\s*,\s*\w+\s*\[[^\]]+\]\s*\)")
    hits = []
    for p in glob.glob(os.path.join(ROOT, "csrc", "kernels", "*")):
        hits += [(os.path.basename(p), m.group(0)) for m in pat.finditer(open(p).read())]
    assert not hits, hits


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_fdot2_repro_isa(tmp_path):
    """The minimal repro's ISA: the bit_cast kernel loads ONE dword per operand and feeds it to all four
    v_dot2 (the miscompile); the pointer-punned kernel loads 16 bytes and uses four distinct dwords.
    If a toolchain update fixes the bit_cast form this test says so (and the note can go)."""
    s = str(tmp_path / "fdot2.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    os.path.join(ROOT, "scripts", "probes", "fdot2_repro.hip"), "-o", s], check=True, capture_output=True)
    text = open(s).read()
    bodies = re.split(r"^_Z\w+:", text, flags=re.M)
    dots = {}
    for name, body in zip(re.findall(r"^(_Z\w+):", text, flags=re.M), bodies[1:]):
        dots[name] = re.findall(r"v_dot2c?_f32_bf16\S*\s+(v\d+),\s*(v\d+),\s*(v\d+)", body)
    bc = next(v for k, v in dots.items() if "bitcast" in k)
    pn = next(v for k, v in dots.items() if "punned" in k)
    assert len(pn) == 4 and len({(a, b) for _, a, b in pn}) == 4, pn
    assert len(bc) == 4
    if len({(a, b) for _, a, b in bc}) == 4:
        pytest.skip("this hipcc compiles the bit_cast form correctly (miscompile fixed)")
    assert len({(a, b) for _, a, b in bc}) == 1, bc  # all four dot products on dword 0
