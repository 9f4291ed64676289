// Skinny projection GEMM for 17..128 rows (decode batches, pipeline micro-batches, short
// prefills): y[M, N] = A[M, K] @ W^T with the fused epilogues of epilogue.h.
//
// Why a third kernel for this regime (profiles/r2_gemm_sk_vs_coop_decode.jsonl): gemv_coop.hip
// stages each A chunk through LDS behind a workgroup barrier and keeps two chunks of weights in
// flight, so a 32..128-row projection advances one chunk per memory round trip (~2 us per
// step, 1.6-4.7 TB/s); gemm_sk.hip's 128-row tiles are in the same place. Here nothing in the
// main loop synchronises between waves:
//  * a workgroup owns TN 16-column tiles and one K range (split s of S); its NWV waves split
//    that range by 32-k step (wave w takes steps w, w + NWV, ...), so every A and W element a
//    workgroup needs is loaded by exactly one of its waves, straight into the MFMA operand
//    registers (A: one 16-B buffer load per lane per 16-row block from the L2-resident
//    activations; W: one 16-B load per lane per packed 1 KiB fragment, non-temporal);
//  * each wave keeps D steps of operands in flight in a register ring (unconditional loads,
//    tail indices clamped to the last step - L1/L2 hits - so every wait is a static count) -
//    4 waves x D x (MB + TN) KiB per CU in flight instead of a chunk per barrier;
//  * the waves' fp32 accumulators are summed once through LDS at the end (a log2(NWV)-round
//    tree), S > 1 splits hand
//    their partial tiles to the last-arriving workgroup of the column group (write-through
//    sc1 stores + relaxed ticket, replay-safe: the last arriver resets the counter) which
//    sums them in fixed split order (deterministic) and runs the epilogue;
//  * NORM: RMSNorm of the A rows fused (weights pre-multiplied by the norm gain,
//    packing.fold_norm): the sum of squares comes from the same A registers.
// Reference op: the four projections of /root/reference/utils/shard_loader.py:66-74.
#include "epilogue.h"

// Timing-only builds (scripts/skinny_ablate.py; outputs garbage): 1 = no A loads, 2 = no weight
// loads, 3 = loads only (no MFMA), 4 = no cross-wave / split reduction and no epilogue, 5 = one
// workgroup barrier after the main loop, then exit, 6 = reduction without the epilogue.
#ifndef LSA_SKINNY_ABLATE
#define LSA_SKINNY_ABLATE 0
#endif

namespace {

template <int MB, int TN, int NWV, int D, int EPI, bool NORM>
__global__ __launch_bounds__(NWV * 64) void skinny_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows, const bf16_raw* __restrict__ wp,
    int M, int N, int K, int S, float eps, EpiArgs ep, float* __restrict__ slab, unsigned* __restrict__ counters) {
  constexpr int NT = NWV * 64;
  constexpr int MR = 16 * MB;
  constexpr int FR = MB * TN;                   // 16x16 output fragments per wave
  constexpr int XB = NWV / 2 * FR * 1024;       // cross-wave tree sum: the upper half's fragments
  constexpr int RS = TN * 16 + 4;               // summed tile row stride (floats, +16 B: banks)
  constexpr int RB = MR * RS * 4;               // summed tile [MR][RS] fp32, row-major
  constexpr int SMEM = XB > RB ? XB : RB;
  static_assert(SMEM <= 128 * 1024, "skinny: LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  __shared__ float s_ssw[NORM ? NWV : 1][MR];
  __shared__ float s_ss[MR];
  __shared__ int s_last;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KT = K >> 5;
  const int G = N / 16 / TN;
  const int g = blockIdx.x % G, s = blockIdx.x / G;
  const int nt0 = g * TN;
  const int kt_lo = s * KT / S, kt_hi = (s + 1) * KT / S;
  const int nk = kt_hi - kt_lo;
  const int n_w = nk > w ? (nk - w + NWV - 1) / NWV : 0;  // this wave's 32-k steps

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0x7fffffff, 0x00020000);
  // A operand of v_mfma_f32_16x16x32_bf16: lane -> row (lane & 15) of the block, k 8*(lane>>4)..+7
  int aoff[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) {
    const int r = min(rb * 16 + (lane & 15), M - 1);  // rows >= M: duplicates, never stored
    aoff[rb] = ((a_rows ? a_rows[r] : r) * ldx + 8 * (lane >> 4)) * 2;
  }
  // W fragment (tile t, step kt) = 1 KiB lane-linear at ((nt0 + t) * KT + kt) KiB
  const int boff = nt0 * KT * 1024 + lane * 16;

  u32x4_t ra[D][MB], rw[D][TN];
  auto issue = [&](u32x4_t (&a)[MB], u32x4_t (&b)[TN], int j) {
    const int kt = kt_lo + w + min(j, n_w - 1) * NWV;
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
      a[rb] = LSA_SKINNY_ABLATE == 1 ? u32x4_t{(unsigned)kt, 0u, 0u, 0u}
                                     : __builtin_amdgcn_raw_buffer_load_b128(xr, aoff[rb], kt * 64, 0);
#pragma unroll
    for (int t = 0; t < TN; ++t)
      b[t] = LSA_SKINNY_ABLATE == 2 ? u32x4_t{(unsigned)kt, 0u, 0u, 0u}
                                    : __builtin_amdgcn_raw_buffer_load_b128(wr, boff + t * KT * 1024, kt * 1024, 2);
  };

  f32x4_t acc[MB][TN];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb)
#pragma unroll
    for (int t = 0; t < TN; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float ssl[MB];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb) ssl[rb] = 0.f;

  if (n_w > 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      issue(ra[d], rw[d], d);
      __builtin_amdgcn_sched_barrier(0);  // stage order = steady-state order: static wait counts
    }
    for (int j0 = 0; j0 < n_w; j0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (j0 + d < n_w) {
          if constexpr (LSA_SKINNY_ABLATE == 3) {
#pragma unroll
            for (int rb = 0; rb < MB; ++rb)
#pragma unroll
              for (int t = 0; t < TN; ++t) acc[rb][t][0] += __uint_as_float(ra[d][rb][0] ^ rw[d][t][1]);
          } else {
#pragma unroll
            for (int rb = 0; rb < MB; ++rb)
#pragma unroll
              for (int t = 0; t < TN; ++t) acc[rb][t] = mfma16(ra[d][rb], rw[d][t], acc[rb][t]);
          }
          if (NORM) {
#pragma unroll
            for (int rb = 0; rb < MB; ++rb) {
              float f[8];
              unpack8(ra[d][rb], f);
#pragma unroll
              for (int e = 0; e < 8; ++e) ssl[rb] += f[e] * f[e];
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // the refill reuses this stage's registers
        issue(ra[d], rw[d], j0 + d + D);  // unconditional (clamped): static wait counts
      }
    }
  }

  if constexpr (LSA_SKINNY_ABLATE == 5) {
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int q = 0; q < TN; ++q) t += acc[rb][q][0] + acc[rb][q][1] + acc[rb][q][2] + acc[rb][q][3];
    if (t == 1.2345f) ep.out[tid] = 0;
    return;
  }
  if constexpr (LSA_SKINNY_ABLATE == 4) {
    float t = 0.f;
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int q = 0; q < TN; ++q) t += acc[rb][q][0] + acc[rb][q][1] + acc[rb][q][2] + acc[rb][q][3];
    if (t == 1.2345f) ep.out[tid] = 0;  // keep the loop live
    return;
  }
  // ---- cross-wave tree sum through LDS (log2(NWV) rounds: the upper half of the remaining waves
  // hands its fragments to the lower half), wave 0 ends with the workgroup's tile
  f32x4_t* xp = reinterpret_cast<f32x4_t*>(smem);
  if (NORM) {
#pragma unroll
    for (int rb = 0; rb < MB; ++rb) {
      float v = ssl[rb];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) s_ssw[w][rb * 16 + lane] = v;
    }
  }
#pragma unroll
  for (int h = NWV / 2; h >= 1; h /= 2) {
    if (w >= h && w < 2 * h) {
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TN; ++t) xp[((w - h) * FR + rb * TN + t) * 64 + lane] = acc[rb][t];
    }
    __syncthreads();
    if (w < h) {
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[rb][t] += xp[(w * FR + rb * TN + t) * 64 + lane];
    }
    __syncthreads();
  }
  float ssum = 0.f;
  if (NORM && tid < MR) {
#pragma unroll
    for (int q = 0; q < NWV; ++q) ssum += s_ssw[q][tid];
  }
  float* red = reinterpret_cast<float*>(smem);  // [MR][RS] (xp is dead)
  auto put_frag = [&](int t, int rb, int ln, f32x4_t v) {
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(rb * 16 + (ln >> 4) * 4 + r) * RS + t * 16 + (ln & 15)] = v[r];
  };
  if (S == 1) {
    if (w == 0) {
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TN; ++t) put_frag(t, rb, lane, acc[rb][t]);
    }
    if (NORM && tid < MR) s_ss[tid] = ssum;
  } else {
    // split hand-off (cdna_hip_programming.md §5 'In-launch split-K reduction', sc1 form), slab
    // fragment-native: [S][N/16 tiles][MB][64 lanes][4] fp32, then [S][G][MR] partial sum(x^2)
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slab, (short)0, 0x7fffffff, 0x00020000);
    const int split_stride = (N / 16) * MR * 16;  // floats
    if (w == 0) {
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TN; ++t)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[rb][t]), sr,
                                                 ((((nt0 + t) * MB + rb) * 64 + lane) * 4) * 4, s * split_stride * 4,
                                                 16 /* sc1 */);
    }
    const int ss_base = S * split_stride;  // floats
    if (NORM && tid < MR)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ssum), sr, ((s * G + g) * MR + tid) * 4, ss_base * 4, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(&counters[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)(S - 1);
    }
    __syncthreads();
    if (!s_last) return;
    // last arriver: the group's TN tiles are one contiguous run of TN*MB*256 floats per split;
    // every thread keeps all its EU x 4 split loads in flight per round trip
    const int gbase = nt0 * MB * 256;
    constexpr int TOT = TN * MB * 64, EU = (TOT + NT - 1) / NT;
    f32x4_t v[EU];
#pragma unroll
    for (int e = 0; e < EU; ++e) v[e] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int q0 = 0; q0 < S; q0 += 4) {
      f32x4_t p[4][EU];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int q = q0 + qq < S ? q0 + qq : 0;
#pragma unroll
        for (int e = 0; e < EU; ++e) {
          const int u = min(e * NT + tid, TOT - 1);
          p[qq][e] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(sr, (gbase + u * 4) * 4,
                                                                                        q * split_stride * 4, 16));
        }
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        if (q0 + qq < S) {
#pragma unroll
          for (int e = 0; e < EU; ++e) v[e] += p[qq][e];
        }
    }
#pragma unroll
    for (int e = 0; e < EU; ++e) {
      const int u = e * NT + tid;
      if (u < TOT) put_frag(u / (MB * 64), (u >> 6) % MB, u & 63, v[e]);
    }
    if (NORM) {
      for (int r = tid; r < MR; r += NT) {
        float t2 = 0.f;
        for (int q = 0; q < S; ++q)
          t2 += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(sr, ((q * G + g) * MR + r) * 4, ss_base * 4, 16));
        s_ss[r] = t2;
      }
    }
    if (tid == 0) __hip_atomic_store(&counters[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();

  if constexpr (LSA_SKINNY_ABLATE == 6) {
    if (red[tid] == 1.2345f) ep.out[tid] = 0;
    return;
  }
  // ---- epilogue: one thread per finished 16-column tile row (SwiGLU: per gate/up tile pair),
  // the TN tiles of one row on consecutive lanes so a wave's stores cover whole output lines
  auto rstd = [&](int mm) -> float { return NORM ? rsqrtf(s_ss[mm] / (float)K + eps) : 1.f; };
  auto load16 = [&](int t, int mm, float r, float* v) {  // rotated quads (LDS banks)
    const float* rp = red + mm * RS + t * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qq = (q + t) & 3;
      const f32x4_t x4 = *reinterpret_cast<const f32x4_t*>(rp + 4 * qq);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * qq + j] = x4[j] * r;
    }
  };
  if constexpr (EPI == EPI_SWIGLU) {
    for (int e = tid; e < (TN / 2) * MR; e += NT) {
      const int tp = e % (TN / 2), mm = e / (TN / 2);
      if (mm >= M) continue;
      const float r = rstd(mm);
      float gg[16], uu[16];
      load16(2 * tp, mm, r, gg);
      load16(2 * tp + 1, mm, r, uu);
#pragma unroll
      for (int j = 0; j < 16; ++j) gg[j] = silu(gg[j]) * uu[j];
      bf16_raw* o = ep.out + (size_t)mm * ep.ldo + (nt0 / 2 + tp) * 16;
      st16(o, pack8(gg));
      st16(o + 8, pack8(gg + 8));
    }
  } else {
    for (int e = tid; e < TN * MR; e += NT) {
      const int t = e % TN, mm = e / TN;
      if (mm >= M) continue;
      float v[16];
      load16(t, mm, rstd(mm), v);
      epi_row16<EPI>(ep, mm, (nt0 + t) * 16, v);
    }
  }
}

template <int MB, int TN, int NWV, int D, int EPI, bool NORM>
int launch(const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp, int M, int N, int K, int S, float eps,
           const EpiArgs& ep, float* slab, unsigned* cnt, hipStream_t s) {
  const int G = N / 16 / TN;
  skinny_kernel<MB, TN, NWV, D, EPI, NORM><<<dim3(G * S), dim3(NWV * 64), 0, s>>>(x, ldx, a_rows, wp, M, N, K, S, eps,
                                                                                  ep, slab, cnt);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

// (mb, tn, nwv, depth) - keep in sync with llm_sharding_amd/ops/packing.py SKINNY_CONFIGS
#define LSA_SKINNY_CONFIGS(X)                                                                              \
  X(2, 4, 4, 4) X(2, 8, 4, 4) X(2, 4, 8, 4) X(2, 2, 8, 4) X(2, 6, 4, 4) X(4, 4, 4, 4) X(4, 2, 8, 4)           \
  X(4, 4, 8, 3) X(4, 8, 4, 3) X(4, 3, 4, 4) X(4, 6, 4, 3) X(8, 4, 4, 3) X(8, 2, 4, 4) X(8, 2, 8, 3)           \
  X(8, 4, 4, 2) X(8, 3, 4, 3) X(8, 6, 4, 2)

template <int EPI, bool NORM>
int dispatch(int mb, int tn, int nwv, int depth, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp,
             int M, int N, int K, int S, float eps, const EpiArgs& ep, float* slab, unsigned* cnt, hipStream_t s) {
#define LSA_C(B, T, W, D)                          \
  if (mb == B && tn == T && nwv == W && depth == D) \
    return launch<B, T, W, D, EPI, NORM>(x, ldx, a_rows, wp, M, N, K, S, eps, ep, slab, cnt, s);
  LSA_SKINNY_CONFIGS(LSA_C)
#undef LSA_C
  return LSA_UNSUPPORTED;
}

}  // namespace

// M <= 128 rows (row blocks mb = 2 / 4 / 8 for M <= 32 / 64 / 128), N % (16 tn) == 0 (SwiGLU:
// tn even), K % 32 == 0, 1 <= sk <= K / 32. Workspace (sk > 1): slab >= sk*N*16*mb +
// sk*(N/16/tn)*16*mb floats, counters >= N/16/tn zero-initialised uint32 (reset in-kernel).
// Epilogues: STORE, RESID, SWIGLU, QKV, each with or without the fused input RMSNorm.
extern "C" int lsa_skinny(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N, int K, int norm,
                          float eps, int epi, const EpiArgs* ep, int tn, int nwv, int depth, int sk, float* slab,
                          long long slab_floats, unsigned* counters, int n_counters, hipStream_t stream) {
  if (M < 1 || M > 128 || K % 32 || K < 32 || ldx < K || ldx % 8 || sk < 1 || sk > K / 32 || tn < 1 || !ep)
    return LSA_BAD_SHAPE;
  if (N % (16 * tn) || (epi == EPI_SWIGLU && tn % 2)) return LSA_BAD_SHAPE;
  const int mb = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
  const long long G = N / 16 / tn;
  if (sk > 1 && (!slab || !counters || n_counters < G || slab_floats < sk * (long long)N * 16 * mb + sk * G * 16 * mb))
    return LSA_BAD_SHAPE;
  if ((long long)N * K * 2 >= (1ll << 31)) return LSA_BAD_SHAPE;  // 32-bit buffer offsets
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
#define LSA_D(E, NM) dispatch<E, NM>(mb, tn, nwv, depth, xx, ldx, a_rows, w, M, N, K, sk, eps, *ep, slab, counters, stream)
  if (norm) {
    switch (epi) {
      case EPI_STORE: return LSA_D(EPI_STORE, true);
      case EPI_RESID: return LSA_D(EPI_RESID, true);
      case EPI_SWIGLU: return LSA_D(EPI_SWIGLU, true);
      case EPI_QKV: return LSA_D(EPI_QKV, true);
      default: return LSA_UNSUPPORTED;
    }
  }
  switch (epi) {
    case EPI_STORE: return LSA_D(EPI_STORE, false);
    case EPI_RESID: return LSA_D(EPI_RESID, false);
    case EPI_SWIGLU: return LSA_D(EPI_SWIGLU, false);
    case EPI_QKV: return LSA_D(EPI_QKV, false);
    default: return LSA_UNSUPPORTED;
  }
#undef LSA_D
}
