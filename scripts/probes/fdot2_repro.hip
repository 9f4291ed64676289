// Minimal test of the round-5 claim that hipcc "folded four __builtin_amdgcn_fdot2_f32_bf16 calls onto
// one dword pair" (profiles/r5_persistent_chain_probe.md). Each lane dots 8 bf16 weights
// with 8 bf16 activations as four v_dot2_f32_bf16 on the four dwords of a 16-byte load, two ways:
//   well-defined: every dword is __builtin_bit_cast to a bf16x2;
//   type-punned:  the 16-byte vector is reinterpreted through a bf16x2 pointer (the probe's form).
// The host compares both with an fp64 reference of the same bf16 products. Build + run:
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/fdot2_repro.hip -o probe_bin/fdot2_repro && probe_bin/fdot2_repro
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void dot_bitcast(const u32x4* w, const u32x4* x, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const u32x4 a = w[i], b = x[i];
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a[k]), __builtin_bit_cast(bf16x2, b[k]), acc,
                                          false);
  out[i] = acc;
}

__global__ void dot_punned(const u32x4* w, const u32x4* x, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 a = w[i], b = x[i];
  const bf16x2* pa = reinterpret_cast<const bf16x2*>(&a);
  const bf16x2* pb = reinterpret_cast<const bf16x2*>(&b);
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = __builtin_amdgcn_fdot2_f32_bf16(pa[k], pb[k], acc, false);
  out[i] = acc;
}

static float bf(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main() {
  const int n = 1 << 20;
  std::vector<unsigned> hw(4 * n), hx(4 * n);
  unsigned s = 7u;
  for (int i = 0; i < 4 * n; ++i) {
    unsigned r[2];
    for (int h = 0; h < 2; ++h) {
      s = s * 1664525u + 1013904223u;
      r[h] = 0x3c00u + ((s >> 9) & 0x7ffu) + ((s >> 31) << 15);  // bf16 in [~0.0078, ~0.06], random sign
    }
    (i & 1 ? hx : hw)[i] = 0;
    hw[i] = r[0] | (r[1] << 16);
    s = s * 1664525u + 1013904223u;
    hx[i] = (0x3f00u + ((s >> 9) & 0xffu)) | ((0x3f00u + ((s >> 17) & 0xffu)) << 16);
  }
  u32x4 *dw, *dx;
  float* dout;
  if (hipMalloc(&dw, 16ull * n) || hipMalloc(&dx, 16ull * n) || hipMalloc(&dout, 4ull * n)) return 2;
  if (hipMemcpy(dw, hw.data(), 16ull * n, hipMemcpyHostToDevice) || hipMemcpy(dx, hx.data(), 16ull * n, hipMemcpyHostToDevice))
    return 2;
  std::vector<float> o(n);
  const char* names[2] = {"bit_cast", "type-punned"};
  int bad_total = 0;
  for (int v = 0; v < 2; ++v) {
    if (v == 0)
      hipLaunchKernelGGL(dot_bitcast, dim3(n / 256), dim3(256), 0, 0, dw, dx, dout);
    else
      hipLaunchKernelGGL(dot_punned, dim3(n / 256), dim3(256), 0, 0, dw, dx, dout);
    if (hipDeviceSynchronize() || hipMemcpy(o.data(), dout, 4ull * n, hipMemcpyDeviceToHost)) return 2;
    int bad = 0, first_only = 0;
    double maxrel = 0.0;
    for (int i = 0; i < n; ++i) {
      double ref = 0.0, ref0 = 0.0, mag = 0.0;  // error relative to sum |products| (no cancellation blow-up)
      for (int k = 0; k < 4; ++k) {
        const unsigned a = hw[4 * i + k], b = hx[4 * i + k];
        const double p0 = (double)bf(a & 0xffff) * bf(b & 0xffff), p1 = (double)bf(a >> 16) * bf(b >> 16);
        ref += p0 + p1;
        mag += std::fabs(p0) + std::fabs(p1);
        if (k == 0) ref0 = 4.0 * (p0 + p1);
      }
      const double rel = std::fabs(o[i] - ref) / (mag + 1e-12);
      if (rel > maxrel) maxrel = rel;
      if (rel > 1e-3) {
        ++bad;
        if (std::fabs(o[i] - ref0) / (mag + 1e-12) < 1e-3) ++first_only;
      }
    }
    printf("%-12s lanes %d, wrong %d (of which = 4 x the first dword pair: %d), max rel err %.2e\n", names[v], n, bad,
           first_only, maxrel);
    bad_total += bad;
  }
  hipFree(dw);
  hipFree(dx);
  hipFree(dout);
  return bad_total ? 1 : 0;
}
