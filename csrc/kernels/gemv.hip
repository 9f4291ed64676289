// Decode projection kernel: y[M, N] = A[M, K] @ W^T with M <= 64 (decode batch), bf16 in,
// fp32 accumulate, fused RMSNorm and fused epilogues (epilogue.h).
//
// Design (MI355X-first, not a translation of the reference's per-op nn.Linear calls in
// /root/reference/utils/shard_loader.py:67-73 / node_worker.py:262):
//  * Batch-1..64 decode is HBM-bound on the weight stream. Every weight byte is read once,
//    16 B/lane, as a whole contiguous 1 KiB MFMA B-fragment from the pre-packed layout
//    (common.h), non-temporal, straight into VGPRs (no LDS round trip).
//  * Two register sets are software-pipelined: the loads of chunk c+1 are in flight while
//    the MFMAs of chunk c run, and every load is unconditional (tail chunks clamp their
//    address and zero their A operand) so hipcc never branches around a load or drains
//    vmcnt to 0 mid-loop (cdna_hip_programming.md §5 'Three .s-level traps' (c)).
//  * The padded A operand (<= 4 x 16 rows) comes from L1/L2; one v_mfma_f32_16x16x32_bf16
//    per (16 cols x 32 k) fragment and row block - MFMA throughput is ~25x the HBM rate.
//  * NW waves per workgroup split K; partial tiles are reduced through LDS and the epilogue
//    runs in natural (row, col) order on the reduced values.
//  * NORM (RMSNorm before the projection): the norm weight is folded into W at load time
//    (W' = W * diag(g)), so A is the raw hidden state; each lane accumulates sum(x^2) of its
//    A fragments during the main loop and the epilogue multiplies by rsqrt(mean + eps).
//    No prologue pass over A and no separate norm launch.
#include "epilogue.h"

namespace {

template <int TN, int MB, int NW, int U, int EPI, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemv_packed_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows,
    const bf16_raw* __restrict__ wp, int M, int N, int K, float eps, EpiArgs ep) {
  constexpr int NTHR = NW * 64;
  constexpr int MR = 16 * MB;  // max rows
  // U = k-fragments per pipeline chunk (two chunks in flight per wave)
  __shared__ float red[NW * TN * MR * 16];
  __shared__ float s_ss[NW][MR];
  __shared__ unsigned long long s_key[MR];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int KT = K >> 5;
  const int nt0 = blockIdx.x * TN;
  const int kq = lane >> 4;
  // Buffer descriptors built from kernel arguments only (wave-uniform, no waterfall loops,
  // cdna_hip_programming.md T8/T20): every load is base(SGPR) + lane voffset + k soffset(SGPR).
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(wp + (size_t)nt0 * KT * 512), (short)0, 0x7fffffff, 0x00020000);
  int xoff[MB];
  bool mvalid[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    const int m = rb * 16 + (lane & 15);
    mvalid[rb] = m < M;
    const int mm = mvalid[rb] ? m : 0;
    xoff[rb] = ((a_rows ? a_rows[mm] : mm) * ldx + kq * 8) * 2;
  }
  if (EPI == EPI_ARGMAX && tid < MR) s_key[tid] = 0ull;

  // Epilogue inputs that do not depend on the result (the residual, the row's cache position and
  // slot), requested before the weight stream so their latency hides under it instead of
  // following it (profiles/r6_gemv_epi_prefetch.md). Only where each thread finishes at most one
  // element (e = tid: every batch-1..16 config with TN * 256 <= NTHR); else loaded in the epilogue.
  constexpr bool PRE = (EPI == EPI_RESID || EPI == EPI_QKV) && TN * MR * 16 <= NTHR;
  // The loads are unconditional (indices clamped into range) and converted only where used: a
  // guarded load made hipcc wait for it (vmcnt(0)) before the main loop.
  bf16_raw pre_r = 0;
  int pre_p = 0, pre_s = 0;
  if constexpr (PRE) {
    const bool in = tid < TN * MR * 16 && ((tid >> 4) % MR) < M;
    const int mm = in ? (tid >> 4) % MR : 0, col = (nt0 + (in ? tid / (MR * 16) : 0)) * 16 + (tid & 15);
    if (EPI == EPI_RESID) {
      pre_r = ep.resid[(size_t)mm * ep.ldr + col];
    } else {
      pre_p = ep.pos[mm];
      pre_s = ep.slot[mm];
    }
  }

  f32x4_t acc[MB][TN];
  float ss[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    ss[rb] = 0.f;
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  // K is split over the NW waves in whole chunks of U fragments (host guarantees KT % U == 0),
  // so no load is ever clamped or predicated.
  const int n_units = KT / U;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int kt_begin = ((wu * n_units) / NW) * U, kt_end = (((wu + 1) * n_units) / NW) * U;
  const int lane16 = lane * 16;
  const u32x4_t zero = {0u, 0u, 0u, 0u};

  auto load = [&](int kt, u32x4_t (&b)[U][TN], u32x4_t (&a)[U][MB]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int t = 0; t < TN; ++t)  // aux 2 = nt: once-read weight stream
        b[u][t] = __builtin_amdgcn_raw_buffer_load_b128(wr, lane16, ((t * KT + kt + u) * 512) * 2, 2);
#pragma unroll
      for (int rb = 0; rb < MB; ++rb) a[u][rb] = __builtin_amdgcn_raw_buffer_load_b128(xr, xoff[rb], (kt + u) * 64, 0);
    }
  };
  auto compute = [&](u32x4_t (&b)[U][TN], u32x4_t (&a)[U][MB]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int rb = 0; rb < MB; ++rb) {
        const u32x4_t av = mvalid[rb] ? a[u][rb] : zero;
        if (NORM) {
          float f[8];
          unpack8(av, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[rb] += f[j] * f[j];
        }
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[rb][t] = mfma16(av, b[u][t], acc[rb][t]);
      }
    }
  };

  if (kt_begin < kt_end) {
    // Every path between two uniform branches is straight-line "issue next chunk, then
    // compute current chunk", so hipcc's counted vmcnt waits only for the current chunk.
    u32x4_t bX[U][TN], aX[U][MB], bY[U][TN], aY[U][MB];
    int kt = kt_begin;
    load(kt, bX, aX);
    for (;;) {
      if (kt + U >= kt_end) {
        compute(bX, aX);
        break;
      }
      load(kt + U, bY, aY);
      compute(bX, aX);
      kt += U;
      if (kt + U >= kt_end) {
        compute(bY, aY);
        break;
      }
      load(kt + U, bX, aX);
      compute(bY, aY);
      kt += U;
    }
  }

  // C layout of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r.
  // red layout: [wave][tile][row 0..MR)[col 0..16)
#pragma unroll
  for (int rb = 0; rb < MB; ++rb)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[((w * TN + t) * MR + rb * 16 + kq * 4 + r) * 16 + (lane & 15)] = acc[rb][t][r];
  if (NORM) {
#pragma unroll
    for (int rb = 0; rb < MB; ++rb) {
      float v = ss[rb];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) s_ss[w][rb * 16 + lane] = v;
    }
  }
  __syncthreads();

  auto rsum = [&](int t, int mm, int n) -> float {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) v += red[((i * TN + t) * MR + mm) * 16 + n];
    return v;
  };
  auto rstd = [&](int mm) -> float {
    if (!NORM) return 1.f;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += s_ss[i][mm];
    return rsqrtf(t / (float)K + eps);
  };

  if (EPI == EPI_SWIGLU) {
    for (int e = tid; e < (TN / 2) * MR * 16; e += NTHR) {
      const int tp = e / (MR * 16), mm = (e >> 4) % MR, n = e & 15;
      if (mm >= M) continue;
      const float r = rstd(mm);
      const float g = rsum(2 * tp, mm, n) * r, u = rsum(2 * tp + 1, mm, n) * r;
      const int col = (nt0 / 2 + tp) * 16 + n;
      ep.out[(size_t)mm * ep.ldo + col] = f2bf(silu(g) * u);
    }
  } else {
    for (int e = tid; e < TN * MR * 16; e += NTHR) {
      const int t = e / (MR * 16), mm = (e >> 4) % MR, n = e & 15;
      if (mm >= M) continue;
      const float r = rstd(mm);
      const float v = rsum(t, mm, n) * r;
      const int col = (nt0 + t) * 16 + n;
      if (EPI == EPI_STORE) {
        ep.out[(size_t)mm * ep.ldo + col] = f2bf(epi_act(ep, v + epi_bias(ep, col)));
      } else if (EPI == EPI_RESID) {
        const float rv = bf2f(PRE ? pre_r : ep.resid[(size_t)mm * ep.ldr + col]);
        ep.out[(size_t)mm * ep.ldo + col] = f2bf(rv + v + epi_bias(ep, col));
      } else if (EPI == EPI_QKV) {
        epi_qkv_store(ep, mm, col, v + epi_bias(ep, col), rsum(t, mm, n ^ 8) * r + epi_bias(ep, col ^ 8),
                      PRE ? pre_p : ep.pos[mm], PRE ? pre_s : ep.slot[mm]);
      } else if (EPI == EPI_ARGMAX) {
        atomicMax(&s_key[mm], argmax_key(v + epi_bias(ep, col), (unsigned)(col + ep.col_offset)));
      }
    }
    if (EPI == EPI_ARGMAX) {
      __syncthreads();
      if (tid < M) atomicMax(&ep.keys[tid], s_key[tid]);
    }
  }
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
