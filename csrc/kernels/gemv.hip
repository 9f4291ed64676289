// Decode projection kernel: y[M, N] = A[M, K] @ W^T with M <= 64 (decode batch), bf16 in,
// fp32 accumulate, fused RMSNorm and fused epilogues (epilogue.h). The body (design notes
// there) lives in gemv_body.h, shared with the fused QKV + attention probe (scripts/probes/qkv_attn.hip).
#include "gemv_body.h"

namespace {

template <int TN, int MB, int NW, int U, int EPI, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemv_packed_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows,
    const bf16_raw* __restrict__ wp, int M, int N, int K, float eps, EpiArgs ep) {
  gemv_packed_body<TN, MB, NW, U, EPI, NORM>(x, ldx, a_rows, wp, M, N, K, eps, ep, blockIdx.x);
}

template <int TN, int MB, int NW, int U, int EPI>
int launch_cfg(bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp, int M,
               int N, int K, float eps, const EpiArgs& ep, hipStream_t s) {
  dim3 grid(N / 16 / TN), block(NW * 64);
  if (norm)
    gemv_packed_kernel<TN, MB, NW, U, EPI, true><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, eps, ep);
  else
    gemv_packed_kernel<TN, MB, NW, U, EPI, false><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, eps, ep);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

// Instantiated (TN, MB, NW, U) configurations. LDS reduction = NW*TN*MB KiB <= 64 KiB;
// VGPRs ~ 2*U*(TN+MB)*4 + 4*TN*MB: U=8 only for the single-tile single-block case.
#define LSA_GEMV_CONFIGS(X)                                                      \
  X(1, 1, 4, 4) X(1, 1, 8, 4) X(1, 1, 16, 4) X(1, 1, 4, 8) X(1, 1, 8, 8)          \
  X(1, 2, 4, 4) X(1, 2, 8, 4) X(1, 2, 16, 2) X(1, 4, 4, 2) X(1, 4, 8, 2)          \
  X(2, 1, 4, 4) X(2, 1, 8, 4) X(2, 1, 16, 2) X(2, 1, 8, 2) X(2, 2, 4, 2)          \
  X(2, 2, 8, 2) X(2, 4, 4, 2) X(2, 4, 8, 2) X(4, 1, 4, 2) X(4, 1, 8, 2)           \
  X(4, 2, 4, 2) X(4, 2, 8, 2) X(4, 4, 4, 2)

template <int EPI>
int launch_epi(int tn, int nw, int u, bool norm, const bf16_raw* x, int ldx, const int* a_rows,
               const bf16_raw* wp, int M, int N, int K, float eps, const EpiArgs& ep, hipStream_t s) {
  const int mb = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_CFG(T, B, W, UU)                                                            \
  if (tn == T && mb == B && nw == W && u == UU) {                                      \
    if constexpr (EPI == EPI_SWIGLU && (T % 2)) return LSA_BAD_SHAPE;                  \
    else return launch_cfg<T, B, W, UU, EPI>(norm, x, ldx, a_rows, wp, M, N, K, eps, ep, s); \
  }
  LSA_GEMV_CONFIGS(LSA_CFG)
#undef LSA_CFG
  return LSA_UNSUPPORTED;
}

}  // namespace

// norm != 0: RMSNorm of the A rows is applied (the norm weight must already be folded into
// the packed weights, see ops/packing.py::fold_norm). tn = 16-col tiles per workgroup,
// nw = waves per workgroup (K split).
extern "C" int lsa_gemv(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N,
                        int K, int norm, float eps, int epi, const EpiArgs* ep, int tn, int nw,
                        int u, hipStream_t stream) {
  if (M < 1 || M > 64 || tn < 1 || u < 1 || N % (16 * tn) || K % 32 || ldx < K) return LSA_BAD_SHAPE;
  if (epi == EPI_SWIGLU && (tn % 2)) return LSA_BAD_SHAPE;
  if ((K >> 5) % u) return LSA_BAD_SHAPE;  // waves take whole chunks (idle waves are fine)
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
  const bool nrm = norm != 0;
  switch (epi) {
    case EPI_STORE: return launch_epi<EPI_STORE>(tn, nw, u, nrm, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    case EPI_RESID: return launch_epi<EPI_RESID>(tn, nw, u, nrm, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    case EPI_SWIGLU: return launch_epi<EPI_SWIGLU>(tn, nw, u, nrm, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    case EPI_QKV: return launch_epi<EPI_QKV>(tn, nw, u, nrm, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    case EPI_ARGMAX: return launch_epi<EPI_ARGMAX>(tn, nw, u, nrm, xx, ldx, a_rows, w, M, N, K, eps, *ep, stream);
    default: return LSA_UNSUPPORTED;
  }
}
