// Probe library (built on the GPU box by scripts/probes/build_gemv_body.sh into build/probes/, never
// part of the product): the decode GEMV compiled THROUGH the shared device-function body
// (gemv_body.h) - the round-4 build that computed wrong rows at (tn 2, mb 4, nw 8, u 2)
// (profiles/r4_gemv_body_regression.md) - with the library's exact C API (lsa_gemv_body ==
// lsa_gemv's signature) so scripts/gemv_det_probe.py can run it beside the library kernel.
// -DLSA_GEMV_CHK: every red[] / s_ss[] index is range-checked; a violation sets *chk_flag.
#include "gemv_body.h"

namespace {

template <int TN, int MB, int NW, int U, int EPI, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemv_body_kernel(const bf16_raw* __restrict__ x, int ldx,
                                                            const int* __restrict__ a_rows,
                                                            const bf16_raw* __restrict__ wp, int M, int N, int K,
                                                            float eps, EpiArgs ep) {
  gemv_packed_body<TN, MB, NW, U, EPI, NORM>(x, ldx, a_rows, wp, M, N, K, eps, ep, blockIdx.x);
}

template <int TN, int MB, int NW, int U, int EPI>
int launch_cfg(bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp, int M, int N, int K,
               float eps, const EpiArgs& ep, hipStream_t s) {
  dim3 grid(N / 16 / TN), block(NW * 64);
  if (norm)
    gemv_body_kernel<TN, MB, NW, U, EPI, true><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, eps, ep);
  else
    gemv_body_kernel<TN, MB, NW, U, EPI, false><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, eps, ep);
  return hipGetLastError() == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}

#define LSA_BODY_CONFIGS(X)                                                      \
  X(1, 1, 4, 4) X(1, 1, 8, 4) X(1, 1, 16, 4) X(1, 1, 4, 8) X(1, 1, 8, 8)          \
  X(1, 2, 4, 4) X(1, 2, 8, 4) X(1, 2, 16, 2) X(1, 4, 4, 2) X(1, 4, 8, 2)          \
  X(2, 1, 4, 4) X(2, 1, 8, 4) X(2, 1, 16, 2) X(2, 1, 8, 2) X(2, 2, 4, 2)          \
  X(2, 2, 8, 2) X(2, 4, 4, 2) X(2, 4, 8, 2) X(4, 1, 4, 2) X(4, 1, 8, 2)           \
  X(4, 2, 4, 2) X(4, 2, 8, 2) X(4, 4, 4, 2)

template <int EPI>
int launch_epi(int tn, int nw, int u, bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp,
               int M, int N, int K, float eps, const EpiArgs& ep, hipStream_t s) {
  const int mb = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_CFG(T, B, W, UU)                                                                  \
  if (tn == T && mb == B && nw == W && u == UU) {                                            \
    if constexpr (EPI == EPI_SWIGLU && (T % 2)) return LSA_BAD_SHAPE;                        \
    else return launch_cfg<T, B, W, UU, EPI>(norm, x, ldx, a_rows, wp, M, N, K, eps, ep, s); \
  }
  LSA_BODY_CONFIGS(LSA_CFG)
#undef LSA_CFG
  return LSA_UNSUPPORTED;
}

}  // namespace

extern "C" int lsa_gemv_body(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N, int K, int norm,
                             float eps, int epi, const EpiArgs* ep, int tn, int nw, int u, hipStream_t stream) {
  if (M < 1 || M > 64 || tn < 1 || u < 1 || N % (16 * tn) || K % 32 || ldx < K || (K >> 5) % u) return LSA_BAD_SHAPE;
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
  switch (epi) {
    case EPI_STORE: return launch_epi<EPI_STORE>(tn, nw, u, norm != 0, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    case EPI_RESID: return launch_epi<EPI_RESID>(tn, nw, u, norm != 0, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    default: return LSA_UNSUPPORTED;
  }
}

#ifdef LSA_GEMV_CHK
extern "C" int lsa_gemv_body_chk(void* host_flag) {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(lsa_gemv_chk_flag), sizeof(v)) != hipSuccess) return LSA_LAUNCH_FAILED;
  *static_cast<unsigned*>(host_flag) = v;
  return LSA_OK;
}
#endif
