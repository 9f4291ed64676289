#!/usr/bin/env python3
"""In-tree native build for llm_sharding_amd.

Produces (git-ignored, but they travel to the GPU box with the gpurun snapshot):
  llm_sharding_amd/_native/liblsa_kernels.so   HIP kernels for gfx950 (hipcc, -O3)
  llm_sharding_amd/_native/liblsa_comm.so      C++ TCP transport (epoll, framed) - no GPU

Incremental: an object is rebuilt only when its source or any header in csrc/ is newer.
Usage: python csrc/build.py [--force] [-j N] [--arch gfx950]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "llm_sharding_amd", "_native")
OBJ = os.path.join(ROOT, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc() -> str:
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else (shutil.which("hipcc") or "hipcc")


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _stale(src: str, obj: str, hdr_mtime: float) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return t < os.path.getmtime(src) or t < hdr_mtime


def _run(cmd: list) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    if r.stdout.strip():
        sys.stderr.write(r.stdout)


def build(force: bool = False, jobs: int = 8, arch: str = "gfx950", verbose: bool = True) -> dict:
    os.makedirs(OUT, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    hdr = _newest_header()
    hipcc = _hipcc()
    kernel_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    comm_srcs = sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    # -fno-slp-vectorize: no packed-FP32 VALU formed from scalar code (the remaining packed FP32
    # comes from explicit vector code). Packed FP32 beside MFMAs is an anti-lever
    # (MI355X_MICROARCH.md, filler prices; batch 1 -4.3 %: profiles/r5_slp_ab.md), and an SLP build
    # of the round-5 shared GEMV body computed wrong rows (profiles/r5_gemv_nondeterminism.md). The
    # SLP and no-SLP libraries differ bitwise only in the decode attention kernels, by FMA
    # contraction (profiles/r6_isa_hazards.md). csrc/isa_audit.py checks the linked library for
    # back-to-back hazards (rules measured on the hardware) after every build.
    hip_flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={arch}", "-Wall",
                 "-Wno-unused-function", "-munsafe-fp-atomics", "-fno-slp-vectorize"]
    # a change of the compile flags rebuilds every object (the flags are part of the stamp)
    stamp = os.path.join(OBJ, "hip_flags.txt")
    if (open(stamp).read() if os.path.exists(stamp) else "") != " ".join(hip_flags):
        force = True
    jobs_list = []
    kobjs = []
    for s in kernel_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        kobjs.append(o)
        if force or _stale(s, o, hdr):
            jobs_list.append([hipcc, *hip_flags, "-c", s, "-o", o])
    cobjs = []
    cxx = shutil.which("g++") or "g++"
    for s in comm_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        cobjs.append(o)
        if force or _stale(s, o, hdr):
            jobs_list.append([cxx, "-O2", "-std=c++17", "-fPIC", "-Wall", "-c", s, "-o", o])
    if verbose and jobs_list:
        print(f"[build] compiling {len(jobs_list)} translation unit(s) for {arch}", file=sys.stderr)
    with cf.ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    out = {}
    klib = os.path.join(OUT, "liblsa_kernels.so")
    # relink also when the set of translation units changed (a removed kernel file must not
    # leave its symbols in the library)
    manifest = os.path.join(OBJ, "liblsa_kernels.objs")
    listed = open(manifest).read() if os.path.exists(manifest) else ""
    if kobjs and (force or not os.path.exists(klib) or listed != "\n".join(kobjs) or
                  os.path.getmtime(klib) < max(os.path.getmtime(o) for o in kobjs)):
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={arch}", *kobjs, "-o", klib])
        with open(manifest, "w") as f:
            f.write("\n".join(kobjs))
    with open(stamp, "w") as f:
        f.write(" ".join(hip_flags))
    audit_stamp = os.path.join(OBJ, "isa_audit.ok")
    if not os.path.exists(audit_stamp) or os.path.getmtime(audit_stamp) < os.path.getmtime(klib):
        sys.path.insert(0, CSRC)
        from isa_audit import audit  # csrc/isa_audit.py
        res = audit(klib, arch)
        if res["code_objects"] == 0:  # an audit that checked nothing must not pass (advisor round 5)
            raise RuntimeError(f"ISA audit of {klib}: no {arch} code object found in the library's offload bundle")
        if res["findings"]:
            raise RuntimeError(f"ISA audit of {klib}: back-to-back hazards {res['by_rule']}, e.g. "
                               f"{res['findings'][:3]} (csrc/isa_audit.py)")
        with open(audit_stamp, "w") as f:
            f.write(f"{res['code_objects']} code objects, {res['packed_fp32_instructions']} packed FP32 (explicit "
                    f"vector code), 0 findings under rules {sorted(res['by_rule'])}\n")
    out["kernels"] = klib
    clib = os.path.join(OUT, "liblsa_comm.so")
    if cobjs and (force or not os.path.exists(clib) or
                  os.path.getmtime(clib) < max(os.path.getmtime(o) for o in cobjs)):
        _run([cxx, "-shared", "-fPIC", *cobjs, "-o", clib, "-lpthread"])
    out["comm"] = clib
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--arch", default=os.environ.get("PYTORCH_ROCM_ARCH", "gfx950"))
    a = ap.parse_args()
    res = build(a.force, a.jobs, a.arch)
    for k, v in res.items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    main()
