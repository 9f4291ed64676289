// The fused projection epilogues of epilogue.h as a standalone pass over a finished bf16
// GEMM output C[M, N] in packed column order (the library GEMM multiplies by the row-major
// image of the packed weights - fused, RoPE-permuted, norm-folded - so RoPE partners and
// gate/up tiles sit exactly where the fused kernels expect them).
//
// Used where the plain GEMM runs on the vendor library (torch.matmul) instead of gemm.hip:
// prefill and decode batches above the 128-row coop-GEMV range, where the library GEMM is ~2x
// the hand-written one (profiles/r1_gemm_vs_hipblaslt.jsonl). The residual adds need no pass
// (beta = 1 in the GEMM); QKV (RoPE + KV-cache append) and SwiGLU do.
//
// One thread per (row, 16-column tile) - per (row, 32-column gate|up pair) for SwiGLU - so a
// wave reads 64 consecutive 32-B runs of a row (coalesced) and stores 16-B runs.
#include "epilogue.h"

namespace {

constexpr int EA_THR = 256;

template <int EPI>
__global__ __launch_bounds__(EA_THR) void epilogue_apply_kernel(const bf16_raw* __restrict__ c, int ldc, int M,
                                                                int N, EpiArgs ep) {
  const int tiles = EPI == EPI_SWIGLU ? N >> 5 : N >> 4;
  const long long idx = (long long)blockIdx.x * EA_THR + threadIdx.x;
  if (idx >= (long long)M * tiles) return;
  const int m = (int)(idx / tiles), t = (int)(idx % tiles);
  const bf16_raw* row = c + (size_t)m * ldc;
  float v[16];
  if (EPI == EPI_SWIGLU) {
    // packed gate_up: 16-column gate tile 2t, then its up tile 2t + 1 -> 16 outputs at 16t
    float g[16], u[16];
    unpack8(ld16(row + 32 * t), g);
    unpack8(ld16(row + 32 * t + 8), g + 8);
    unpack8(ld16(row + 32 * t + 16), u);
    unpack8(ld16(row + 32 * t + 24), u + 8);
    epi_bias16(ep, 32 * t, g);
    epi_bias16(ep, 32 * t + 16, u);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = silu(g[j]) * u[j];
    bf16_raw* o = ep.out + (size_t)m * ep.ldo + 16 * t;
    st16(o, pack8(v));
    st16(o + 8, pack8(v + 8));
    return;
  }
  unpack8(ld16(row + 16 * t), v);
  unpack8(ld16(row + 16 * t + 8), v + 8);
  epi_row16<EPI>(ep, m, 16 * t, v);
}

}  // namespace

extern "C" int lsa_epilogue_apply(const void* c, int ldc, int M, int N, int epi, const EpiArgs* ep,
                                  hipStream_t stream) {
  if (M < 1 || N % 16 || ldc < N || ldc % 8 || !ep || !ep->out) return LSA_BAD_SHAPE;
  if (epi == EPI_SWIGLU && N % 32) return LSA_BAD_SHAPE;
  if (epi == EPI_RESID && !ep->resid) return LSA_BAD_SHAPE;
  if (epi == EPI_QKV && (!ep->k_cache || !ep->v_cache || !ep->slot || !ep->pos)) return LSA_BAD_SHAPE;
  const long long work = (long long)M * (epi == EPI_SWIGLU ? N / 32 : N / 16);
  const int grid = (int)((work + EA_THR - 1) / EA_THR);
  const bf16_raw* C = static_cast<const bf16_raw*>(c);
  switch (epi) {
    case EPI_STORE: epilogue_apply_kernel<EPI_STORE><<<grid, EA_THR, 0, stream>>>(C, ldc, M, N, *ep); break;
    case EPI_RESID: epilogue_apply_kernel<EPI_RESID><<<grid, EA_THR, 0, stream>>>(C, ldc, M, N, *ep); break;
    case EPI_SWIGLU: epilogue_apply_kernel<EPI_SWIGLU><<<grid, EA_THR, 0, stream>>>(C, ldc, M, N, *ep); break;
    case EPI_QKV: epilogue_apply_kernel<EPI_QKV><<<grid, EA_THR, 0, stream>>>(C, ldc, M, N, *ep); break;
    default: return LSA_UNSUPPORTED;
  }
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}
