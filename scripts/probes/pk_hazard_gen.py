#!/usr/bin/env python3
"""Generates and builds scripts/probes/pk_hazard_probe.hip: a hardware test of which VALU
writer -> packed-FP32 reader pairs need wait states on MI355X (gfx950), the ground truth behind
csrc/isa_audit.py's rule.

Every case is one inline-asm sequence (the compiler's hazard recognizer does not look inside an
asm statement, so the instructions issue exactly as written): registers v40-v47 are set up, a
WRITER instruction updates v40 (or v41), GAP instructions follow, then a READER consumes the
v[40:41] pair; the result is compared bitwise with the same sequence run with 16 wait states
between writer and reader. A mismatch means the reader saw the register before the write.
Output (one line per case): writer, gap, reader, mismatching lanes / lanes tested, for one wave
per SIMD and for 8 waves per SIMD.

usage: python scripts/probes/pk_hazard_gen.py   (writes + builds probe_bin/pk_hazard_probe)"""
import itertools
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "scripts", "probes", "pk_hazard_probe.hip")
BIN = os.path.join(ROOT, "probe_bin", "pk_hazard_probe")  # git-ignored; travels with gpurun

WRITERS = {
    "valu32_lo": "v_add_f32 v40, v40, %[e]",
    "valu32_hi": "v_add_f32 v41, v41, %[e]",
    "vop3_fma_lo": "v_fma_f32 v40, v40, %[e], %[e]",
    "dpp_lo": "v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
    "trans_lo": "v_exp_f32 v40, %[e]",
    "cvt_pk_lo": "v_cvt_pk_bf16_f32 v40, %[e], %[e]",
    "and_hi": "v_and_b32 v41, 0xffff0000, %[e]",
    "mov_lo": "v_mov_b32 v40, %[e]",
    "pk_add": "v_pk_add_f32 v[40:41], v[40:41], v[42:43]",
    "pk_fma_acc": "v_pk_fma_f32 v[40:41], v[42:43], v[42:43], v[40:41]",
    # the round-5 GEMV site: both halves of the pair updated by 32-bit FMAs, then the packed read
    "fma_lo_hi": "v_fma_f32 v40, v42, v42, v40\\n v_fma_f32 v41, v43, v43, v41",
    "rsq_lo": "v_rsq_f32 v40, %[e]",
}
READERS = {
    "pk_add": "v_pk_add_f32 v[44:45], v[40:41], v[42:43]",
    "pk_mul": "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]",
    "pk_fma_src0": "v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]",
    "pk_fma_src2": "v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]",
    "pk_mov": "v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]",
    "add_f32": "v_add_f32 v44, v40, v42",
    "dpp_read": "v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
}
GAPS = {
    "0": "",
    "nop0": "s_nop 0",
    "valu1": "v_mov_b32 v48, v49",
    "nop1": "s_nop 1",
    "valu2": "v_mov_b32 v48, v49\\n v_mov_b32 v50, v49",
}
SAFE = "s_nop 7\\n s_nop 7"


def seq(w, g, r):
    return ("v_mov_b32 v40, %[a]\\n v_mov_b32 v41, %[b]\\n v_mov_b32 v42, %[c]\\n v_mov_b32 v43, %[d]\\n"
            " v_mov_b32 v46, %[d]\\n v_mov_b32 v47, %[c]\\n v_mov_b32 v44, 0\\n v_mov_b32 v45, 0\\n"
            " v_mov_b32 v49, %[a]\\n s_nop 7\\n s_nop 7\\n"
            f" {w}\\n {g}\\n {r}\\n s_nop 7\\n v_mov_b32 %[o0], v44\\n v_mov_b32 %[o1], v45\\n")


def gen() -> list:
    cases = list(itertools.product(WRITERS, GAPS, READERS))
    out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <cstring>', '']
    out.append('typedef float f32x4 __attribute__((ext_vector_type(4)));')
    out.append('typedef unsigned u32x4 __attribute__((ext_vector_type(4)));')
    out.append('typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));')
    out.append('#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50"')
    for ci, (w, g, r) in enumerate(cases):
        hz = seq(WRITERS[w], GAPS[g], READERS[r])
        sf = seq(WRITERS[w], SAFE, READERS[r])
        out.append(f"""__global__ void case_{ci}(const float* __restrict__ in, unsigned* __restrict__ bad, int iters, int partner) {{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (partner && (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 1)) {{  // MFMA-issuing partner wave
    f32x4 acc = {{0.f, 0.f, 0.f, 0.f}};
    bf16x8 x = __builtin_bit_cast(bf16x8, u32x4{{(unsigned)i, 3u, 5u, 7u}});
    for (int it = 0; it < iters * 16; ++it) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, acc, 0, 0, 0);
    bad[i] = acc[0] == 1234.5f ? 1u : 0u;
    return;
  }}
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {{
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("{hz}" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("{sf}" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }}
  bad[i] = nb;
}}""")
    out.append("typedef void (*KFn)(const float*, unsigned*, int, int);")
    out.append("static const KFn KS[] = {" + ", ".join(f"case_{i}" for i in range(len(cases))) + "};")
    out.append("static const char* NAMES[] = {" + ", ".join(f'"{w} {g} {r}"' for w, g, r in cases) + "};")
    out.append(f"""int main() {{
  const int N = 4096, ITERS = 64;
  std::vector<float> h(N);
  unsigned s = 12345u;
  for (int i = 0; i < N; ++i) {{ s = s * 1664525u + 1013904223u; h[i] = ((s >> 8) & 0xffff) / 4096.0f - 8.0f + 0.001f * i; }}
  float* din; unsigned* dbad;
  hipMalloc(&din, N * 4);
  const int MAXT = 256 * 8 * 256;
  hipMalloc(&dbad, MAXT * 4);
  hipMemcpy(din, h.data(), N * 4, hipMemcpyHostToDevice);
  std::vector<unsigned> hb(MAXT);
  // (blocks, threads, partner): one wave per SIMD (1024 x 64), 8 waves per SIMD (1024 x 512), and
  // 8 waves per SIMD where every other wave issues MFMAs instead (the GEMV's two-waves-per-SIMD
  // neighbourhood)
  const int cfg[3][3] = {{{{1024, 64, 0}}, {{1024, 512, 0}}, {{1024, 512, 1}}}};
  for (int c = 0; c < {len(cases)}; ++c) {{
    unsigned long long tot[3] = {{0, 0, 0}}, tested[3] = {{0, 0, 0}};
    for (int k = 0; k < 3; ++k) {{
      const int nb = cfg[k][0], nt = cfg[k][1];
      hipLaunchKernelGGL(KS[c], dim3(nb), dim3(nt), 0, 0, din, dbad, ITERS, cfg[k][2]);
      if (hipDeviceSynchronize() != hipSuccess) {{ printf("case %d failed\\n", c); return 2; }}
      hipMemcpy(hb.data(), dbad, (size_t)nb * nt * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < nb * nt; ++i) tot[k] += hb[i];
      tested[k] = 2ull * nb * nt * ITERS / (cfg[k][2] ? 2 : 1);
      if (cfg[k][2]) {{ tot[k] = 0; for (int q = 0; q < nb * nt; ++q) if (((q % nt) >> 6) % 2 == 0) tot[k] += hb[q]; }}
    }}
    printf("%-40s 1w/SIMD %llu/%llu  8w/SIMD %llu/%llu  4w+4mfma/SIMD %llu/%llu\\n", NAMES[c], tot[0], tested[0], tot[1],
           tested[1], tot[2], tested[2]);
  }}
  hipFree(din); hipFree(dbad);
  return 0;
}}""")
    with open(SRC, "w") as f:
        f.write("\n".join(out) + "\n")
    return cases


if __name__ == "__main__":
    cases = gen()
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "--offload-arch=gfx950", SRC, "-o", BIN], check=True)
    print(f"{len(cases)} cases -> {BIN}")
