// Instruction-fetch cost at kernel launch on MI355X: one wave per CU executes an unrolled block of
// NOPS independent VALU ops (8 accumulators, issue-bound when the code is cached) REPS times
// (outer loop, not unrolled). The first pass fetches the block cold, later passes run from the
// instruction cache: time(REPS=1) - (time(REPS=2) - time(REPS=1)) - empty launch = cold-fetch
// cost of the block. Diagnostic only (scripts/icache_probe.py builds and runs it).
#include <hip/hip_runtime.h>

template <int NOPS>
__global__ __launch_bounds__(64) void block(float* out, float a, int reps) {
  float x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3f + k;
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int i = 0; i < NOPS; ++i) x[i & 7] = __builtin_fmaf(x[i & 7], a, 0.5f + (i >> 3) * 1e-6f);
  }
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) t += x[k];
  if (t == 12345.f) out[threadIdx.x] = t;
}

extern "C" int run_icache(int reps, int nops, float* out, int grid, hipStream_t s) {
#define L(N)                                                         \
  if (nops == N) {                                                   \
    block<N><<<grid, 64, 0, s>>>(out, 1.0001f, reps);                \
    return hipGetLastError() == hipSuccess ? 0 : 2;                  \
  }
  L(8) L(512) L(1024) L(2048) L(3072)
#undef L
  return 1;
}
