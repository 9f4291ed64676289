// Per-CU operand-load throughput on MI355X from an L2-resident buffer (every workgroup re-reads
// the same 1 MiB): (0) LDS-DMA (global_load_lds_dwordx4) into a 128 KiB LDS ring, (1) dwordx4
// loads into VGPRs, (2) half of each. 512-thread workgroups, one per CU, DEPTH instructions in
// flight per wave. Diagnostic only (scripts/load_path_probe.py builds and runs it).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) unsigned int u4;

template <int MODE, int DEPTH>
__global__ __launch_bounds__(512) void probe(const unsigned char* __restrict__ src, int iters, unsigned* sink,
                                             long long span) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[128 * 1024];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  u4 acc = {0u, 0u, 0u, 0u};
  // span == 0: each wave walks its own 64 KiB window of the 1 MiB buffer (L2-resident);
  // span > 0: each wave streams through its own 1/2048 slice of a span-byte buffer (MALL / HBM)
  const long long slice = span > 0 ? span / 2048 : 65536;
  const unsigned char* base = src + (span > 0 ? (long long)(blockIdx.x * 8 + w) * slice
                                              : (long long)((blockIdx.x * 8 + w) % 16) * 65536);
  const int nkb = (int)(slice / 1024);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const long long off = (long long)((it * DEPTH + d) % nkb) * 1024 + lane * 16;
      if (MODE == 0 || (MODE == 2 && (d & 1) == 0)) {
        __builtin_amdgcn_global_load_lds(base + off, (__attribute__((address_space(3))) void*)(lds + (w * 16 + (d % 16)) * 1024),
                                         16, 0, 0);
      } else {
        u4 v = *reinterpret_cast<const u4*>(base + off);
        acc ^= v;
      }
    }
    if (MODE == 1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DEPTH / 2) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}

extern "C" int run_probe(int mode, int depth, const void* src, int grid, int iters, unsigned* sink, long long span,
                         hipStream_t s) {
  const auto* p = static_cast<const unsigned char*>(src);
#define L(M, D) probe<M, D><<<grid, 512, 0, s>>>(p, iters, sink, span)
  if (mode == 0 && depth == 8) L(0, 8);
  else if (mode == 0 && depth == 16) L(0, 16);
  else if (mode == 1 && depth == 8) L(1, 8);
  else if (mode == 1 && depth == 16) L(1, 16);
  else if (mode == 2 && depth == 8) L(2, 8);
  else if (mode == 2 && depth == 16) L(2, 16);
  else if (mode == 0 && depth == 32) L(0, 32);
  else if (mode == 1 && depth == 32) L(1, 32);
  else return 1;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
