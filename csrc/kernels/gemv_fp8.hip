// W8A16 decode projection: y[M, N] = A[M, K] @ (Q[N, K] * scale[N])^T for M <= 64, with OCP
// FP8 e4m3 weights (the ModelSharder's FP8 shard format, per-output-channel scales; MI355X /
// gfx950 uses the OCP encoding natively), bf16 activations, fp32 accumulation and the same
// fused RMSNorm / epilogues as gemv.hip.
//
// Decode is bound by the weight stream, so halving the weight bytes halves the HBM time:
//  * packed layout Wq[nt][kt/2][lane][16 B]: one 16-B non-temporal buffer load per lane brings
//    TWO consecutive 32-k MFMA B fragments (bytes 0-7 and 8-15, element order as pack_b);
//  * v_cvt_scalef32_pk_bf16_fp8 turns 2 fp8 into 2 bf16 (4 per fragment), so the bf16
//    v_mfma_f32_16x16x32_bf16 does the math - activations are never quantised;
//  * the per-channel scale is applied once, in fp32, in the epilogue (a lane's B fragment
//    belongs to a single output column, but scaling after accumulation is exact and free).
// Same register double-buffering / whole-chunk wave split / LDS reduction as gemv.hip.
#include "epilogue.h"

namespace {

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// 8 fp8 (two dwords) -> 8 bf16 (u32x4)
LSA_DEVICE u32x4_t fp8x8_to_bf16(unsigned lo, unsigned hi) {
  u32x4_t r;
  r[0] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, false));
  r[1] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, true));
  r[2] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, false));
  r[3] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, true));
  return r;
}

// U2 = 16-B weight loads (= 2 k-fragments each) per pipeline chunk and tile
template <int TN, int MB, int NW, int U2, int EPI, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemv_fp8_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows,
    const unsigned char* __restrict__ wq, const float* __restrict__ wscale, int M, int N, int K, float eps,
    EpiArgs ep) {
  constexpr int NTHR = NW * 64;
  constexpr int MR = 16 * MB;
  constexpr int U = 2 * U2;  // k-fragments per chunk
  __shared__ float red[NW * TN * MR * 16];
  __shared__ float s_ss[NW][MR];
  __shared__ unsigned long long s_key[MR];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int KT = K >> 5, KT2 = KT >> 1;
  const int nt0 = blockIdx.x * TN;
  const int kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(wq + (size_t)nt0 * KT2 * 1024), (short)0, 0x7fffffff, 0x00020000);
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

  f32x4_t acc[MB][TN];
  float ss[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    ss[rb] = 0.f;
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  const int n_units = KT / U;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int kt_begin = ((wu * n_units) / NW) * U, kt_end = (((wu + 1) * n_units) / NW) * U;
  const int lane16 = lane * 16;
  const u32x4_t zero = {0u, 0u, 0u, 0u};

  auto load = [&](int kt, u32x4_t (&b)[U2][TN], u32x4_t (&a)[U][MB]) {
#pragma unroll
    for (int u = 0; u < U2; ++u)
#pragma unroll
      for (int t = 0; t < TN; ++t)  // nt: once-read weight stream
        b[u][t] = __builtin_amdgcn_raw_buffer_load_b128(wr, lane16, (t * KT2 + (kt >> 1) + u) * 1024, 2);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int rb = 0; rb < MB; ++rb) a[u][rb] = __builtin_amdgcn_raw_buffer_load_b128(xr, xoff[rb], (kt + u) * 64, 0);
  };
  auto compute = [&](u32x4_t (&b)[U2][TN], u32x4_t (&a)[U][MB]) {
#pragma unroll
    for (int u2 = 0; u2 < U2; ++u2) {
      u32x4_t bf[2][TN];
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        bf[0][t] = fp8x8_to_bf16(b[u2][t][0], b[u2][t][1]);
        bf[1][t] = fp8x8_to_bf16(b[u2][t][2], b[u2][t][3]);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int rb = 0; rb < MB; ++rb) {
          const u32x4_t av = mvalid[rb] ? a[2 * u2 + h][rb] : zero;
          if (NORM) {
            float f[8];
            unpack8(av, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss[rb] += f[j] * f[j];
          }
#pragma unroll
          for (int t = 0; t < TN; ++t) acc[rb][t] = mfma16(av, bf[h][t], acc[rb][t]);
        }
    }
  };

  if (kt_begin < kt_end) {
    u32x4_t bX[U2][TN], aX[U][MB], bY[U2][TN], aY[U][MB];
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
    return v * wscale[(nt0 + t) * 16 + n];
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
      ep.out[(size_t)mm * ep.ldo + (nt0 / 2 + tp) * 16 + n] = f2bf(silu(g) * u);
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
        ep.out[(size_t)mm * ep.ldo + col] = f2bf(bf2f(ep.resid[(size_t)mm * ep.ldr + col]) + v + epi_bias(ep, col));
      } else if (EPI == EPI_QKV) {
        epi_qkv_store(ep, mm, col, v + epi_bias(ep, col), rsum(t, mm, n ^ 8) * r + epi_bias(ep, col ^ 8), ep.pos[mm],
                      ep.slot[mm]);
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

template <int TN, int MB, int NW, int U2, int EPI>
int launch_cfg(bool norm, const bf16_raw* x, int ldx, const int* a_rows, const unsigned char* wq, const float* ws,
               int M, int N, int K, float eps, const EpiArgs& ep, hipStream_t s) {
  dim3 grid(N / 16 / TN), block(NW * 64);
  if (norm)
    gemv_fp8_kernel<TN, MB, NW, U2, EPI, true><<<grid, block, 0, s>>>(x, ldx, a_rows, wq, ws, M, N, K, eps, ep);
  else
    gemv_fp8_kernel<TN, MB, NW, U2, EPI, false><<<grid, block, 0, s>>>(x, ldx, a_rows, wq, ws, M, N, K, eps, ep);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

// (TN, MB, NW, U2): U2 16-B fp8 loads per tile per chunk (= 2*U2 k-fragments)
#define LSA_FP8_CONFIGS(X)                                                                     \
  X(1, 1, 4, 2) X(1, 1, 8, 2) X(1, 1, 4, 4) X(2, 1, 4, 2) X(2, 1, 8, 2) X(4, 1, 4, 1)           \
  X(1, 2, 4, 2) X(1, 2, 8, 2) X(2, 2, 4, 1) X(2, 2, 8, 1) X(1, 4, 4, 1) X(1, 4, 8, 1) X(2, 4, 4, 1) \
  X(2, 4, 8, 1)

template <int EPI>
int launch_epi(int tn, int nw, int u2, bool norm, const bf16_raw* x, int ldx, const int* a_rows,
               const unsigned char* wq, const float* ws, int M, int N, int K, float eps, const EpiArgs& ep,
               hipStream_t s) {
  const int mb = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
#define LSA_CFG(T, B, W, UU)                                                                       \
  if (tn == T && mb == B && nw == W && u2 == UU) {                                                \
    if constexpr (EPI == EPI_SWIGLU && (T % 2)) return LSA_BAD_SHAPE;                             \
    else return launch_cfg<T, B, W, UU, EPI>(norm, x, ldx, a_rows, wq, ws, M, N, K, eps, ep, s);   \
  }
  LSA_FP8_CONFIGS(LSA_CFG)
#undef LSA_CFG
  return LSA_UNSUPPORTED;
}

// Dequantise packed fp8 (Wq[nt][kt/2][lane][16]) into packed bf16 (Wp[nt][kt][lane][8]) with the
// per-row scale: used to run prefill / >64-row batches through the bf16 GEMM / coop kernels
// from one layer-sized scratch buffer when the weights are kept in fp8.
__global__ void dequant_fp8_packed_kernel(const unsigned char* __restrict__ wq, const float* __restrict__ wscale,
                                          bf16_raw* __restrict__ wp, int NT, int KT2) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // one 16-B fp8 load = 2 fragments
  if (i >= (size_t)NT * KT2 * 64) return;
  const int lane = (int)(i & 63);
  const size_t blk = i >> 6;  // nt * KT2 + kt2
  const int nt = (int)(blk / KT2), kt2 = (int)(blk % KT2);
  const u32x4_t q = *reinterpret_cast<const u32x4_t*>(wq + i * 16);
  const float sc = wscale[nt * 16 + (lane & 15)];
  for (int h = 0; h < 2; ++h) {
    const u32x4_t b = fp8x8_to_bf16(q[2 * h], q[2 * h + 1]);
    float f[8];
    unpack8(b, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= sc;
    const size_t frag = ((size_t)nt * (2 * KT2) + 2 * kt2 + h) * 64 + lane;
    *reinterpret_cast<u32x4_t*>(wp + frag * 8) = pack8(f);
  }
}

}  // namespace

extern "C" int lsa_gemv_fp8(const void* x, int ldx, const int* a_rows, const void* wq, const float* wscale, int M,
                            int N, int K, int norm, float eps, int epi, const EpiArgs* ep, int tn, int nw, int u2,
                            hipStream_t stream) {
  if (M < 1 || M > 64 || tn < 1 || u2 < 1 || N % (16 * tn) || K % 64 || ldx < K || !wscale) return LSA_BAD_SHAPE;
  if (epi == EPI_SWIGLU && (tn % 2)) return LSA_BAD_SHAPE;
  if ((K >> 5) % (2 * u2)) return LSA_BAD_SHAPE;
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const unsigned char* w = static_cast<const unsigned char*>(wq);
  const bool nrm = norm != 0;
  switch (epi) {
    case EPI_STORE: return launch_epi<EPI_STORE>(tn, nw, u2, nrm, xx, ldx, a_rows, w, wscale, M, N, K, eps, *ep, stream);
    case EPI_RESID: return launch_epi<EPI_RESID>(tn, nw, u2, nrm, xx, ldx, a_rows, w, wscale, M, N, K, eps, *ep, stream);
    case EPI_SWIGLU: return launch_epi<EPI_SWIGLU>(tn, nw, u2, nrm, xx, ldx, a_rows, w, wscale, M, N, K, eps, *ep, stream);
    case EPI_QKV: return launch_epi<EPI_QKV>(tn, nw, u2, nrm, xx, ldx, a_rows, w, wscale, M, N, K, eps, *ep, stream);
    case EPI_ARGMAX: return launch_epi<EPI_ARGMAX>(tn, nw, u2, nrm, xx, ldx, a_rows, w, wscale, M, N, K, eps, *ep, stream);
    default: return LSA_UNSUPPORTED;
  }
}

extern "C" int lsa_dequant_fp8_packed(const void* wq, const float* wscale, void* wp, int N, int K, hipStream_t stream) {
  if (N % 16 || K % 64) return LSA_BAD_SHAPE;
  const int NT = N / 16, KT2 = K / 64;
  const size_t n = (size_t)NT * KT2 * 64;
  dequant_fp8_packed_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(
      static_cast<const unsigned char*>(wq), wscale, static_cast<bf16_raw*>(wp), NT, KT2);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}
