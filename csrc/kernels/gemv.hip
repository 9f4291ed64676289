// Decode projection kernel: y[M, N] = A[M, K] @ W^T with M <= 64 (decode batch), bf16 in,
// fp32 accumulate, fused RMSNorm prologue and fused epilogues (epilogue.h).
//
// Design (MI355X-first, not a translation of the reference's per-op nn.Linear calls in
// /root/reference/utils/shard_loader.py:67-73 / node_worker.py:262):
//  * Batch-1..16 decode is HBM-bound on the weight stream. Every weight byte is read once,
//    16 B/lane, as a whole contiguous 1 KiB MFMA B-fragment from the pre-packed layout
//    (common.h), non-temporal, straight into VGPRs (no LDS round trip).
//  * The padded 16-row A operand comes from L1/L2 (the activations are tiny and shared by
//    every workgroup); rows >= M are zero and never loaded.
//  * One v_mfma_f32_16x16x32_bf16 per (16 cols x 32 k) fragment and 16-row block: MFMA
//    throughput is ~25x the HBM rate here, so M=1 costs the same as M=16; up to 4 row
//    blocks (M <= 64) share each streamed weight fragment.
//  * 8 waves per workgroup split K; partial 16x16 tiles are reduced through LDS and the
//    epilogue runs in natural (row, col) order on the reduced values.
//  * NORM: the workgroup computes rstd of its A rows itself (A rows are L2-resident), so the
//    input/post-attention/final RMSNorm never needs its own launch.
#include "epilogue.h"

namespace {

constexpr int NWAVE = 8;
constexpr int NTHR = NWAVE * LSA_WAVE;

template <int TN, int MB, int EPI, bool NORM>
__global__ __launch_bounds__(NTHR) void gemv_packed_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows,
    const bf16_raw* __restrict__ wp, int M, int N, int K,
    const bf16_raw* __restrict__ norm_w, float eps, EpiArgs ep) {
  constexpr int MR = 16 * MB;  // max rows
  __shared__ float red[NWAVE * TN * MB * 256];
  __shared__ float s_part[NWAVE][MR];
  __shared__ float s_rstd[MR];
  __shared__ unsigned long long s_key[MR];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int KT = K >> 5;
  const int nt0 = blockIdx.x * TN;
  const int kq = lane >> 4;
  const bf16_raw* xrow[MB];
  bool mvalid[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    const int m = rb * 16 + (lane & 15);
    mvalid[rb] = m < M;
    xrow[rb] = x + (size_t)(mvalid[rb] ? (a_rows ? a_rows[m] : m) : 0) * ldx;
  }

  if (EPI == EPI_ARGMAX && tid < MR) s_key[tid] = 0ull;

  if (NORM) {
    for (int r = 0; r < M; ++r) {
      const bf16_raw* xr = x + (size_t)(a_rows ? a_rows[r] : r) * ldx;
      float s = 0.f;
      for (int c = tid; c < (K >> 3); c += NTHR) {
        float f[8];
        unpack8(ld16(xr + c * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += f[j] * f[j];
      }
      s = wave_sum(s);
      if (lane == 0) s_part[w][r] = s;
    }
    __syncthreads();
    if (tid < M) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < NWAVE; ++i) t += s_part[i][tid];
      s_rstd[tid] = rsqrtf(t / (float)K + eps);
    }
    __syncthreads();
  }
  float rs[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) rs[rb] = (NORM && mvalid[rb]) ? s_rstd[rb * 16 + (lane & 15)] : 1.f;

  auto load_a = [&](int kt, int rb) -> u32x4_t {
    u32x4_t v = {0u, 0u, 0u, 0u};
    if (mvalid[rb]) {
      const int k = kt * 32 + kq * 8;
      v = ld16(xrow[rb] + k);
      if (NORM) {
        float f[8], g[8];
        unpack8(v, f);
        unpack8(ld16(norm_w + k), g);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = f[j] * rs[rb] * g[j];
        v = pack8(f);
      }
    }
    return v;
  };

  f32x4_t acc[MB][TN];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb)
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int kt_begin = (w * KT) / NWAVE, kt_end = ((w + 1) * KT) / NWAVE;
  const bf16_raw* wb = wp + (size_t)nt0 * KT * 512 + lane * 8;
  constexpr int U = (MB * TN >= 4) ? 2 : 4;
  int kt = kt_begin;
  for (; kt + U <= kt_end; kt += U) {
    u32x4_t b[U][TN];
    u32x4_t a[U][MB];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < TN; ++t) b[u][t] = ld16_nt(wb + ((size_t)t * KT + kt + u) * 512);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int rb = 0; rb < MB; ++rb) a[u][rb] = load_a(kt + u, rb);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[rb][t] = mfma16(a[u][rb], b[u][t], acc[rb][t]);
  }
  for (; kt < kt_end; ++kt) {
    u32x4_t b[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) b[t] = ld16_nt(wb + ((size_t)t * KT + kt) * 512);
#pragma unroll
    for (int rb = 0; rb < MB; ++rb) {
      const u32x4_t a = load_a(kt, rb);
#pragma unroll
      for (int t = 0; t < TN; ++t) acc[rb][t] = mfma16(a, b[t], acc[rb][t]);
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
  __syncthreads();

  auto rsum = [&](int t, int mm, int n) -> float {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NWAVE; ++i) v += red[((i * TN + t) * MR + mm) * 16 + n];
    return v;
  };

  if (EPI == EPI_SWIGLU) {
    for (int e = tid; e < (TN / 2) * MR * 16; e += NTHR) {
      const int tp = e / (MR * 16), mm = (e >> 4) % MR, n = e & 15;
      if (mm >= M) continue;
      const float g = rsum(2 * tp, mm, n), u = rsum(2 * tp + 1, mm, n);
      const int col = (nt0 / 2 + tp) * 16 + n;
      ep.out[(size_t)mm * ep.ldo + col] = f2bf(silu(g) * u);
    }
  } else {
    for (int e = tid; e < TN * MR * 16; e += NTHR) {
      const int t = e / (MR * 16), mm = (e >> 4) % MR, n = e & 15;
      if (mm >= M) continue;
      const float v = rsum(t, mm, n);
      const int col = (nt0 + t) * 16 + n;
      if (EPI == EPI_STORE) {
        ep.out[(size_t)mm * ep.ldo + col] = f2bf(v);
      } else if (EPI == EPI_RESID) {
        ep.out[(size_t)mm * ep.ldo + col] = f2bf(bf2f(ep.resid[(size_t)mm * ep.ldr + col]) + v);
      } else if (EPI == EPI_QKV) {
        epi_qkv_store(ep, mm, col, v, rsum(t, mm, n ^ 8));
      } else if (EPI == EPI_ARGMAX) {
        atomicMax(&s_key[mm], argmax_key(v, (unsigned)(col + ep.col_offset)));
      }
    }
    if (EPI == EPI_ARGMAX) {
      __syncthreads();
      if (tid < M) atomicMax(&ep.keys[tid], s_key[tid]);
    }
  }
}

template <int TN, int MB, int EPI>
int launch_tn(bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp, int M,
              int N, int K, const bf16_raw* nw, float eps, const EpiArgs& ep, hipStream_t s) {
  const int NT = N / 16;
  dim3 grid(NT / TN), block(NTHR);
  if (norm)
    gemv_packed_kernel<TN, MB, EPI, true><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, nw, eps, ep);
  else
    gemv_packed_kernel<TN, MB, EPI, false><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, nw, eps, ep);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

template <int EPI>
int launch_epi(int tn, bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp,
               int M, int N, int K, const bf16_raw* nw, float eps, const EpiArgs& ep, hipStream_t s) {
  const int mb = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_TN_MB(T, B) \
  if (tn == T && mb == B) return launch_tn<T, B, EPI>(norm, x, ldx, a_rows, wp, M, N, K, nw, eps, ep, s);
  if (EPI != EPI_SWIGLU) {
    LSA_TN_MB(1, 1) LSA_TN_MB(1, 2) LSA_TN_MB(1, 4)
  }
  LSA_TN_MB(2, 1) LSA_TN_MB(2, 2) LSA_TN_MB(2, 4)
  LSA_TN_MB(4, 1) LSA_TN_MB(4, 2)
#undef LSA_TN_MB
  return LSA_UNSUPPORTED;
}

}  // namespace

extern "C" int lsa_gemv(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N,
                        int K, const void* norm_w, float eps, int epi, const EpiArgs* ep, int tn,
                        hipStream_t stream) {
  if (M < 1 || M > 64 || N % (16 * tn) || K % 32 || ldx < K) return LSA_BAD_SHAPE;
  if (M > 32 && tn > 2) return LSA_UNSUPPORTED;
  if (epi == EPI_SWIGLU && (tn % 2)) return LSA_BAD_SHAPE;
  const bool norm = norm_w != nullptr;
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
  const bf16_raw* nw = static_cast<const bf16_raw*>(norm_w);
  switch (epi) {
    case EPI_STORE: return launch_epi<EPI_STORE>(tn, norm, xx, ldx, a_rows, w, M, N, K, nw, eps, *ep, stream);
    case EPI_RESID: return launch_epi<EPI_RESID>(tn, norm, xx, ldx, a_rows, w, M, N, K, nw, eps, *ep, stream);
    case EPI_SWIGLU: return launch_epi<EPI_SWIGLU>(tn, norm, xx, ldx, a_rows, w, M, N, K, nw, eps, *ep, stream);
    case EPI_QKV: return launch_epi<EPI_QKV>(tn, norm, xx, ldx, a_rows, w, M, N, K, nw, eps, *ep, stream);
    case EPI_ARGMAX: return launch_epi<EPI_ARGMAX>(tn, norm, xx, ldx, a_rows, w, M, N, K, nw, eps, *ep, stream);
    default: return LSA_UNSUPPORTED;
  }
}
