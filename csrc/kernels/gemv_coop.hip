// Cooperative split-K projection for 17..128 rows (decode batches, short prefills): y[M, N] = A[M, K] @ W^T.
//
// Why (profiles/r1_gemv_o_proj_pmc.txt): in gemv.hip every workgroup re-reads all of A from
// L2 (waves split K inside the workgroup, so A is never shared); at M >= 32 the L1->L2 request
// count grows ~5x over M = 1 at equal HBM bytes and issue stalls dominate. Here
//  * the NW waves of a workgroup own NW*TNW different 16-column tiles and SHARE each A chunk
//    (M rows x 64 k) staged once through LDS (XOR-swizzled 16-B chunks, double-buffered,
//    register-prefetched one chunk ahead, one barrier per chunk);
//  * every wave streams only its own packed weight fragments (buffer loads, nt), prefetched
//    one chunk ahead in registers;
//  * K is split over SK workgroups; each writes fp32 partial tiles (+ partial sum(x^2) for the
//    fused RMSNorm) to a slab with write-through (sc1) stores, and the last-arriving workgroup
//    of a column group (arrival counter, sc1 loads: the sc1 form of cdna_hip_programming.md
//    §5 'In-launch split-K reduction' / §6 Guideline 16) sums the SK slabs in a fixed order
//    (deterministic) and runs the fused epilogue. The arrival counter
//    is reset by the last arriver, so the kernel is replay-safe inside hipGraphs.
#include "epilogue.h"

#include <utility>

// Timing-only builds (scripts/coop_phases.py; outputs garbage): 1 = exit after the main loop,
// 2 = exit after the k-group / split reduction (no epilogue), 3 = epilogue without its global
// stores, 4 = epilogue stores of constants (no LDS reads, no math).
#ifndef LSA_COOP_ABLATE
#define LSA_COOP_ABLATE 0
#endif

// Diagnostic build only (-DLSA_COOP_STAMPS, scripts/coop_stamps.py): per-workgroup
// s_memrealtime stamps (100 MHz) at the phase boundaries, written by thread 0 to a buffer nothing
// else reads: 0 start, 1 main loop done (wave 0), 2 all waves done, 3 k-group sum done, 4 slab
// stored, 5 ticket drawn, 6 (last arriver) slabs summed, 7 tile in LDS, 8 epilogue done.
#ifdef LSA_COOP_STAMPS
__device__ unsigned long long* g_coop_stamps;
#define LSA_CSTAMP(slot)                                                                                      \
  do {                                                                                                       \
    if (threadIdx.x == 0 && g_coop_stamps) g_coop_stamps[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LSA_CSTAMP(slot) \
  do {                   \
  } while (0)
#endif

namespace {

// f(integral_constant<S>) for S = 0, 1, ... while f returns true
template <int... S, typename F>
LSA_DEVICE bool coop_static_all(std::integer_sequence<int, S...>, F&& f) {
  return (f(std::integral_constant<int, S>{}) && ...);
}

// A tile [MR][KC] bf16 in LDS, 16-B chunks XOR-swizzled so that the 16 lanes of one
// ds_read_b128 pass (16 consecutive rows, same logical chunk) hit all 64 banks: rows of >= 16
// chunks (>= 256 B) XOR with row & 15; 128-B rows pair up two rows per 256-B bank line, so
// they XOR with (row >> 1) & 7 (measured: the old row & 7 swizzle was 2-way conflicted,
// ~3 conflict cycles per LDS instruction in profiles/r1_coop_pmc_m64.txt).
template <int KC>
LSA_DEVICE int a_off(int row, int c16) {
  constexpr int C16 = KC / 8;
  const int sw = C16 >= 16 ? (row & 15) : ((row >> 1) & (C16 - 1));
  return row * (KC * 2) + ((c16 ^ sw) << 4);
}

// 8 OCP fp8 e4m3 (two dwords) -> 8 bf16 (v_cvt_scalef32_pk_bf16_fp8, gfx950)
LSA_DEVICE u32x4_t fp8x8_to_bf16(unsigned lo, unsigned hi) {
  u32x4_t r;
  r[0] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, false));
  r[1] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, true));
  r[2] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, false));
  r[3] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, true));
  return r;
}

// KW > 1: the workgroup holds KW groups of NW waves; group kg streams the kg-th contiguous
// part of the split's K chunks for the SAME NW*TNW tiles (A chunks of every group staged
// side by side in LDS), and the groups' fp32 partials are summed through LDS before the
// epilogue. More waves (bytes in flight) per workgroup at the same column grouping: the
// decode projections have too few 16-column tiles to give every CU a workgroup of 8+ waves.
// D: register-ring depth of the main loop (prefetch distance D-1 chunks for both operands).
template <int MB, int TNW, int NW, int KF, int KW, int D, int EPI, bool NORM, bool FP8>
__global__ __launch_bounds__(NW * KW * 64) void gemv_coop_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows, const bf16_raw* __restrict__ wp,
    int M, int N, int K, int SK, float eps, EpiArgs ep, float* __restrict__ slab, unsigned* __restrict__ counters,
    const float* __restrict__ wscale) {
  constexpr int NTHR = NW * KW * 64;
  constexpr int KC = 32 * KF;                   // k per chunk (KF MFMA k-fragments)
  constexpr int C16 = KC / 8;                   // 16-B pieces per A row
  constexpr int MR = 16 * MB;
  constexpr int TG = NW * TNW;                  // 16-col tiles per workgroup
  constexpr int ABUF = MR * KC * 2;             // bytes per A chunk of one k-group
  constexpr int ABUFT = KW * ABUF;              // bytes per A buffer (all k-groups)
  constexpr int RS = 20;                        // reduction tile row stride (floats): 16 + 4 pad
  constexpr int RED = TG * MR * RS * 4;         // fp32 reduction tile [TG][MR][RS]
  constexpr int XRED = (KW - 1) * TG * MB * 64 * 16;  // k-group partials, fragment-native
  constexpr int SMEM0 = (2 * ABUFT > RED ? 2 * ABUFT : RED);
  constexpr int SMEM = (SMEM0 > XRED ? SMEM0 : XRED);
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  __shared__ float s_ss[MR];
  __shared__ int s_last;
  __shared__ unsigned long long s_key[MR];

  const int tid = threadIdx.x, lane = tid & 63;
  LSA_CSTAMP(0);
  const int wt = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int w = wt % NW, kg = wt / NW;          // tile wave within the k-group, k-group
  const int KT = K >> 5;
  // SK == 0 ("ragged"): no K split; the column tiles (gate / up PAIRS for SwiGLU) are dealt out
  // evenly to the grid's workgroups (one per CU), tcnt <= TG each - a tile count that is not a
  // multiple of TG still fills every CU (Llama-2-7B gate_up at 128 rows: 1,376 tiles = 172 groups
  // of 8 on 172 CUs, or 5-6 tiles on each of 256). Waves past tcnt re-stream the last tile
  // (nothing of theirs is stored). Otherwise: column group g of TG tiles, K split s of SK.
  const bool ragged = SK == 0;
  const int SKe = ragged ? 1 : SK;
  int g = 0, s = 0, tlo, tcnt;
  if (ragged) {
    constexpr int P = EPI == EPI_SWIGLU ? 2 : 1;
    const int units = N / 16 / P;
    tlo = P * (int)(((long long)blockIdx.x * units) / gridDim.x);
    tcnt = P * (int)((((long long)blockIdx.x + 1) * units) / gridDim.x) - tlo;
  } else {
    const int G = N / 16 / TG;                  // column groups
    g = blockIdx.x % G;
    s = blockIdx.x / G;
    tlo = g * TG;
    tcnt = TG;
  }
  const int G = ragged ? 1 : N / 16 / TG;
  const int nt0 = tlo + (w * TNW < tcnt - TNW ? w * TNW : tcnt - TNW);  // this wave's first tile
  const int nch_all = KT / KF;                  // KC-k chunks; split s owns [c_lo, c_hi)
  const int c_lo = s * nch_all / SKe, c_hi = (s + 1) * nch_all / SKe;
  // k-group q owns chunks [q*nchunk, (q+1)*nchunk) of the split (host: divisible by KW)
  const int kt0 = c_lo * KF, nchunk = (c_hi - c_lo) / KW;

  // ---- A staging: thread -> (row + i*RSTEP, 16-B chunk) fixed for all chunks, one load per
  // k-group per i
  // A loads per thread per chunk and k-group; with 3- or 6-wave workgroups the tile does not
  // split evenly and the last load's row can fall past the tile (in_tile: not stored, not summed)
  constexpr int LPT = (MR * C16 + NTHR - 1) / NTHR;
  constexpr bool A_EXACT = LPT * NTHR == MR * C16;
  static_assert(NTHR % C16 == 0, "a thread keeps its 16-B column for every load");
  constexpr int RSTEP = NTHR / C16;
  const int arow = tid / C16, ac16 = tid % C16;
  auto in_tile = [&](int i) { return A_EXACT || arow + i * RSTEP < MR; };
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
  int a_voff[LPT];
  bool a_valid[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int r = arow + i * RSTEP;
    a_valid[i] = r < M && in_tile(i);
    a_voff[i] = ((a_valid[i] ? (a_rows ? a_rows[r] : r) : 0) * ldx + ac16 * 8) * 2;
  }
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0x7fffffff, 0x00020000);
  const int lane16 = lane * 16;
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  float ss[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) ss[i] = 0.f;

  // Epilogue inputs that do not depend on the result, requested early so their round trip hides
  // under other work instead of following the reduction (profiles/r6_gemv_epi_prefetch.md):
  // QKV: the rows' pos / slot here (2 VGPRs per row); RESID: the residual after the main loop
  // (8 VGPRs per row, beside the split hand-off). Thread tid finishes rows e = tid + i * NTHR,
  // i < EPT; the loads are unconditional with clamped indices (a guarded load made hipcc wait).
  constexpr int EPT = (TG * MR + NTHR - 1) / NTHR;
  constexpr bool PRE_R = EPI == EPI_RESID, PRE_Q = EPI == EPI_QKV;
  u32x4_t pre_r[PRE_R ? EPT : 1][2];
  int pre_p[PRE_Q ? EPT : 1], pre_s[PRE_Q ? EPT : 1];
  if constexpr (PRE_Q) {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NTHR, mm = e % MR < M ? e % MR : 0;
      pre_p[i] = ep.pos[mm];
      pre_s[i] = ep.slot[mm];
    }
  }

  struct AV { u32x4_t v[KW][LPT]; };
  auto load_a = [&](int c) -> AV {
    AV a;
#pragma unroll
    for (int q = 0; q < KW; ++q)
#pragma unroll
      for (int i = 0; i < LPT; ++i)
        a.v[q][i] = __builtin_amdgcn_raw_buffer_load_b128(xr, a_voff[i], (kt0 * 32 + (q * nchunk + c) * KC) * 2, 0);
    return a;
  };
  auto store_a = [&](int buf, const AV& a_in, float count) {  // count: 0 for clamped duplicates
#pragma unroll
    for (int q = 0; q < KW; ++q)
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        // rows >= M were loaded from row 0 (valid memory): zero them here
        const u32x4_t av = a_valid[i] ? a_in.v[q][i] : zero;
        if (NORM) {
          float f[8];
          unpack8(av, f);
          float t = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) t += f[j] * f[j];
          ss[i] += count * t;
        }
        if (in_tile(i)) *reinterpret_cast<u32x4_t*>(smem + buf * ABUFT + q * ABUF + a_off<KC>(arow + i * RSTEP, ac16)) = av;
      }
  };
  // B fragments: bf16 -> one 16-B load per k-fragment; FP8 (W8A16, packed as in gemv_fp8.hip)
  // -> one 16-B load per PAIR of k-fragments, converted to bf16 in registers right before the
  // MFMAs (the per-row scale is applied in fp32 in the epilogue)
  constexpr int BL = FP8 ? KF / 2 : KF;
  auto load_b = [&](int c, u32x4_t (&b)[BL][TNW]) {
#pragma unroll
    for (int p = 0; p < BL; ++p)
#pragma unroll
      for (int t = 0; t < TNW; ++t) {
        if constexpr (FP8)
          b[p][t] = __builtin_amdgcn_raw_buffer_load_b128(
              wr, lane16, ((nt0 + t) * (KT >> 1) + ((kt0 + (kg * nchunk + c) * KF) >> 1) + p) * 1024, 2);
        else
          b[p][t] = __builtin_amdgcn_raw_buffer_load_b128(
              wr, lane16, (((nt0 + t) * KT + kt0 + (kg * nchunk + c) * KF + p) * 512) * 2, 2);
      }
  };

  f32x4_t acc[MB][TNW];
#pragma unroll
  for (int rb = 0; rb < MB; ++rb)
#pragma unroll
    for (int t = 0; t < TNW; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // The A fragments of a group of GK k-fragments (GK*MB <= 16 ds_read_b128) are all issued
  // before the group's MFMAs (sched_barrier): with one wave per SIMD nothing else hides LDS
  // latency, and the default schedule waited lgkmcnt on a fresh read before every MFMA.
  constexpr int GK = (16 / MB) < KF ? (16 / MB > 0 ? 16 / MB : 1) : KF;
  static_assert(KF % GK == 0, "k-fragment groups must tile the chunk");
  auto compute = [&](int buf, u32x4_t (&b)[BL][TNW]) {
    const unsigned char* base = smem + buf * ABUFT + kg * ABUF;
#pragma unroll
    for (int k0 = 0; k0 < KF; k0 += GK) {
      u32x4_t af[GK][MB];
#pragma unroll
      for (int j = 0; j < GK; ++j)
#pragma unroll
        for (int rb = 0; rb < MB; ++rb)
          af[j][rb] = *reinterpret_cast<const u32x4_t*>(
              base + a_off<KC>(rb * 16 + (lane & 15), (k0 + j) * 4 + (lane >> 4)));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < GK; ++j) {
        const int kf = k0 + j;
        u32x4_t bk[TNW];
#pragma unroll
        for (int t = 0; t < TNW; ++t) {
          if constexpr (FP8)
            bk[t] = (kf & 1) ? fp8x8_to_bf16(b[kf >> 1][t][2], b[kf >> 1][t][3])
                             : fp8x8_to_bf16(b[kf >> 1][t][0], b[kf >> 1][t][1]);
          else
            bk[t] = b[kf][t];
        }
#pragma unroll
        for (int rb = 0; rb < MB; ++rb)
#pragma unroll
          for (int t = 0; t < TNW; ++t) acc[rb][t] = mfma16(af[j][rb], bk[t], acc[rb][t]);
      }
    }
  };

  {
    // B (HBM weights) is consumed straight from registers, A (L2-resident activations) is
    // written to one of 2 LDS buffers one chunk before use. Loads are unconditional (tail
    // chunk indices clamped, duplicates hit L2) so every s_waitcnt is a static count, never
    // vmcnt(0).
    // D-deep register rings for both operands (prefetch distance D-1 chunks): A and W of one
    // chunk are issued together, so the counted wait for A(c+1) never drains a W prefetch
    // issued after it.
    u32x4_t bw[D][BL][TNW];
    AV aw[D];
    const int last = nchunk - 1;
    auto clampc = [&](int c) { return c < last ? c : last; };
    coop_static_all(std::make_integer_sequence<int, D - 1>{}, [&](auto sc) {
      constexpr int S = decltype(sc)::value;
      aw[S] = load_a(clampc(S));
      load_b(clampc(S), bw[S]);
      return true;
    });
    store_a(0, aw[0], 1.f);
    __syncthreads();
    // step c (ring slot S = c % D): prefetch chunk c+D-1 into slot (c-1) % D, compute chunk c
    // from (LDS c&1, W slot S), then publish A(c+1) into LDS.
    for (int c = 0;;) {
      const bool more = coop_static_all(std::make_integer_sequence<int, D>{}, [&](auto sc) {
        constexpr int S = decltype(sc)::value, SN = (S + D - 1) % D, S1 = (S + 1) % D;
        aw[SN] = load_a(clampc(c + D - 1));
        load_b(clampc(c + D - 1), bw[SN]);
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetches ahead of this chunk's MFMAs
        compute(c & 1, bw[S]);
        __builtin_amdgcn_sched_barrier(0);
        store_a((c + 1) & 1, aw[S1], c < last ? 1.f : 0.f);
        __syncthreads();
        return ++c <= last;
      });
      if (!more) break;
    }
  }

  // row sum(x^2) of this split: the C16 threads of a row are consecutive lanes
  if (NORM) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
#pragma unroll
      for (int o = 1; o < C16; o <<= 1) ss[i] += __shfl_xor(ss[i], o, 64);
    }
  }
  LSA_CSTAMP(1);
  __syncthreads();  // all waves done with the A buffers: smem becomes the reduction tile
  LSA_CSTAMP(2);
  if constexpr (LSA_COOP_ABLATE == 1) {
    float t = 0.f;
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int q = 0; q < TNW; ++q) t += acc[rb][q][0] + acc[rb][q][1] + acc[rb][q][2] + acc[rb][q][3];
    if (t == 1.2345f) ep.out[tid] = 0;  // keep the loop live
    return;
  }
  if constexpr (PRE_R) {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NTHR;
      const bool in = e < tcnt * MR && e % MR < M;
      const bf16_raw* rr = ep.resid + (size_t)(in ? e % MR : 0) * ep.ldr + (tlo + (in ? e / MR : 0)) * 16;
      pre_r[i][0] = ld16(rr);
      pre_r[i][1] = ld16(rr + 8);
    }
  }
  if constexpr (KW > 1) {
    // k-groups 1..KW-1 hand their partial tiles to group 0 (fragment-native, 16 B per lane)
    f32x4_t* xp = reinterpret_cast<f32x4_t*>(smem);  // [KW-1][TG][MB][64]
    if (kg > 0) {
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TNW; ++t) xp[(((kg - 1) * TG + w * TNW + t) * MB + rb) * 64 + lane] = acc[rb][t];
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int q = 1; q < KW; ++q)
#pragma unroll
        for (int rb = 0; rb < MB; ++rb)
#pragma unroll
          for (int t = 0; t < TNW; ++t) acc[rb][t] += xp[(((q - 1) * TG + w * TNW + t) * MB + rb) * 64 + lane];
    }
    __syncthreads();
  }
  LSA_CSTAMP(3);
  float* red = reinterpret_cast<float*>(smem);  // [TG][MR][RS]
  if (SKe == 1 || EPI == EPI_PARTIAL) {  // EPI_PARTIAL: every split stores its own fp32 tile
    if (kg == 0)
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int t = 0; t < TNW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          red[((w * TNW + t) * MR + rb * 16 + (lane >> 4) * 4 + r) * RS + (lane & 15)] = acc[rb][t][r];
    if (NORM && ac16 == 0) {
#pragma unroll
      for (int i = 0; i < LPT; ++i)
        if (in_tile(i)) s_ss[arow + i * RSTEP] = ss[i];
    }
  } else {
    // Split-K hand-off (cdna_hip_programming.md §5 'In-launch split-K reduction', sc1 form):
    // every partial is stored write-through (sc1, 16-B stores), every storing wave drains its
    // stores, the workgroup barriers, one lane takes a relaxed agent-scope ticket; the
    // workgroup that draws SK-1 reads all slabs with sc1 loads. No L2 writeback (release) or
    // invalidate (acquire) is needed in this form.
    // Slab layout, fragment-native so each lane stores its 4 accumulators as one 16-B word:
    //   [SK][N/16 tiles][MB][64 lanes][4]  fp32, then [SK][G][MR] partial sum(x^2).
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slab, (short)0, 0x7fffffff, 0x00020000);
    const int split_stride = (N / 16) * MR * 16;  // floats
    if (kg == 0)
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int t = 0; t < TNW; ++t)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[rb][t]), sr,
                                               ((((nt0 + t) * MB + rb) * 64 + lane) * 4) * 4, s * split_stride * 4,
                                               16 /* sc1 */);
    const int ss_base = SK * split_stride;  // floats
    if (NORM && ac16 == 0) {
#pragma unroll
      for (int i = 0; i < LPT; ++i)
        if (in_tile(i))
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ss[i]), sr, ((s * G + g) * MR + arow + i * RSTEP) * 4,
                                                ss_base * 4, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    LSA_CSTAMP(4);
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(&counters[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)(SK - 1);
    }
    __syncthreads();
    LSA_CSTAMP(5);
    if (!s_last) return;
    // Last arriver: sum the SK slabs in fixed split order (deterministic). The group's region
    // is one contiguous run of TG*MB*256 floats per split; every thread keeps E4 16-B loads x
    // 4 splits in flight per round trip (cross-XCD reads: batching them keeps this short).
    constexpr int E4 = TG * MB * 64 / NTHR;
    static_assert(E4 * NTHR == TG * MB * 64, "combine tiling");
    const int gbase = g * TG * MB * 256;  // floats
    f32x4_t sum[E4];
#pragma unroll
    for (int j = 0; j < E4; ++j) sum[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int q0 = 0; q0 < SK; q0 += 4) {
      f32x4_t v[4][E4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int q = q0 + qq < SK ? q0 + qq : 0;
#pragma unroll
        for (int j = 0; j < E4; ++j)
          v[qq][j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                     sr, (gbase + (j * NTHR + tid) * 4) * 4, q * split_stride * 4, 16));
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        if (q0 + qq < SK)
#pragma unroll
          for (int j = 0; j < E4; ++j) sum[j] += v[qq][j];
    }
#pragma unroll
    for (int j = 0; j < E4; ++j) {
      const int u = j * NTHR + tid;
      const int tl = u / (MB * 64), rb = (u >> 6) % MB, ln = u & 63;
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(tl * MR + rb * 16 + (ln >> 4) * 4 + r) * RS + (ln & 15)] = sum[j][r];
    }
    if (NORM) {
      for (int r = tid; r < MR; r += NTHR) {  // NTHR may be < MR (single-wave workgroups)
        float t2 = 0.f;
        for (int q = 0; q < SK; ++q)
          t2 += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(sr, ((q * G + g) * MR + r) * 4, ss_base * 4, 16));
        s_ss[r] = t2;
      }
    }
    LSA_CSTAMP(6);
    if (tid == 0) __hip_atomic_store(&counters[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (LSA_COOP_ABLATE == 2) {
    __syncthreads();
    if (red[tid] == 1.2345f) ep.out[tid] = 0;
    return;
  }
  if (EPI == EPI_ARGMAX)
    for (int r = tid; r < MR; r += NTHR) s_key[r] = 0ull;
  __syncthreads();

  LSA_CSTAMP(7);
  auto rstd = [&](int mm) -> float { return NORM ? rsqrtf(s_ss[mm] / (float)K + eps) : 1.f; };
  const int ntg0 = tlo;
  // rows RS = 20 floats apart: the 16 rows one ds_read_b128 lane group reads start 20 banks
  // apart (all 64 banks, conflict-free) with the quads in static order - a row-dependent quad
  // rotation made v[] dynamically indexed (~1,200 v_cndmask per epilogue, 2.5-5.5 us per launch)
  auto load16 = [&](int t, int mm, float r, float* v) {
    const float* rp = red + (t * MR + mm) * RS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4_t x4 = *reinterpret_cast<const f32x4_t*>(rp + 4 * q);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * q + j] = x4[j] * r;
    }
    if (FP8) {
      const float* sp = wscale + (ntg0 + t) * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4_t s4 = *reinterpret_cast<const f32x4_t*>(sp + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * q + j] *= s4[j];
      }
    }
  };
  if (EPI == EPI_SWIGLU) {
    // gate tile 2tp / up tile 2tp+1 -> 16 outputs per thread, two 16-B stores
    for (int e = tid; e < (tcnt / 2) * MR; e += NTHR) {
      const int tp = e / MR, mm = e % MR;
      if (mm >= M) continue;
      const float r = rstd(mm);
      float gg[16], uu[16];
      load16(2 * tp, mm, r, gg);
      load16(2 * tp + 1, mm, r, uu);
#pragma unroll
      for (int j = 0; j < 16; ++j) gg[j] = silu(gg[j]) * uu[j];
      bf16_raw* o = ep.out + (size_t)mm * ep.ldo + (ntg0 / 2 + tp) * 16;
      st16(o, pack8(gg));
      st16(o + 8, pack8(gg + 8));
    }
  } else {
    // one thread per finished 16-column tile row (epilogue.h epi_row16); rows e = tid + i * NTHR
    // (static i: the prefetched inputs stay in registers)
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NTHR;
      if (e >= tcnt * MR) break;
      const int t = e / MR, mm = e % MR;
      if (mm >= M) continue;
      if constexpr (LSA_COOP_ABLATE == 4) {
        bf16_raw* o = ep.out + (size_t)mm * ep.ldo + (ntg0 + t) * 16;
        st16(o, u32x4_t{0u, 0u, 0u, 0u});
        st16(o + 8, u32x4_t{0u, 0u, 0u, 0u});
        continue;
      }
      const float r = rstd(mm);
      const int c0 = (ntg0 + t) * 16;
      float v[16];
      load16(t, mm, r, v);
      if (EPI == EPI_ARGMAX) {
        epi_bias16(ep, c0, v);
        atomicMax(&s_key[mm], argmax_key16(v, (unsigned)(c0 + ep.col_offset)));
      } else if constexpr (EPI == EPI_PARTIAL) {
        // fp32 partial of split s at ((float*)out)[s][M][ldo] (lsa_resid_rmsnorm_partials adds
        // the splits to the residual stream in fixed order)
        float* po = reinterpret_cast<float*>(ep.out) + ((size_t)s * M + mm) * ep.ldo + c0;
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4_t*>(po + 4 * q) = f32x4_t{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      } else if constexpr (LSA_COOP_ABLATE == 3) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += v[j];
        if (t == 1.2345f) ep.out[mm] = 0;
      } else if constexpr (PRE_R) {
        epi_bias16(ep, c0, v);
        epi_resid_row16(ep, mm, c0, v, pre_r[i][0], pre_r[i][1]);
      } else if constexpr (PRE_Q) {
        epi_bias16(ep, c0, v);
        epi_qkv_row16p(ep, mm, c0, v, pre_p[i], pre_s[i]);
      } else {
        epi_row16<EPI>(ep, mm, c0, v);
      }
    }
    if (EPI == EPI_ARGMAX) {
      __syncthreads();
      for (int r = tid; r < M; r += NTHR) atomicMax(&ep.keys[r], s_key[r]);
    }
  }
  LSA_CSTAMP(8);
}

// compute units of the current device (the ragged mode's grid: one workgroup per CU)
int n_cu() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    cached[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return cached[dev];
}

template <int MB, int TNW, int NW, int KF, int KW, int D, int EPI, bool FP8>
int launch(bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp, int M, int N, int K, int SK, float eps,
           const EpiArgs& ep, float* slab, unsigned* cnt, const float* wscale, hipStream_t s) {
  const int G = N / 16 / (NW * TNW);
  dim3 grid(SK ? G * SK : n_cu()), block(NW * KW * 64);
  if (norm)
    gemv_coop_kernel<MB, TNW, NW, KF, KW, D, EPI, true, FP8><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, SK, eps, ep, slab, cnt, wscale);
  else
    gemv_coop_kernel<MB, TNW, NW, KF, KW, D, EPI, false, FP8><<<grid, block, 0, s>>>(x, ldx, a_rows, wp, M, N, K, SK, eps, ep, slab, cnt, wscale);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

// (mb, tnw, nw, kf, kw, d). nw = 3 / 6: one workgroup per CU for 768-tile projections (Llama-2-7B
// qkv) with no split at all; nw = 1: one tile per workgroup (4096-column projections). d = 4
// (a deeper ring) where it measured faster: the long unsplit K ranges of gate_up / lm_head and
// 32-row qkv / down (profiles/r4_coop_depth_probe.jsonl); d = 3 everywhere else (deeper rings
// slowed the split configs).
#define LSA_COOP_CONFIGS(X) \
  X(2, 1, 8, 8, 1, 3) X(4, 1, 8, 8, 1, 3) X(2, 1, 8, 4, 1, 3) X(4, 1, 8, 4, 1, 3) X(2, 2, 8, 4, 1, 3) X(4, 2, 8, 4, 1, 3) \
  X(2, 2, 4, 4, 1, 3) X(4, 2, 4, 4, 1, 3) X(8, 1, 8, 4, 1, 3) X(8, 1, 8, 2, 1, 3) X(8, 2, 4, 2, 1, 3) X(2, 1, 4, 4, 1, 3) \
  X(4, 1, 4, 4, 1, 3) X(2, 1, 4, 8, 1, 3) X(8, 1, 4, 2, 1, 3) \
  X(2, 1, 4, 8, 2, 3) X(4, 1, 4, 4, 2, 3) X(4, 1, 4, 8, 2, 3) X(4, 1, 8, 4, 2, 3) X(4, 2, 4, 4, 2, 3) X(8, 1, 4, 2, 2, 3) \
  X(8, 1, 4, 4, 2, 3) X(4, 1, 4, 4, 4, 3) X(4, 1, 2, 4, 2, 3) X(4, 1, 2, 4, 1, 3) X(2, 1, 2, 4, 2, 3) X(8, 1, 2, 2, 2, 3) \
  X(8, 1, 3, 2, 1, 3) X(8, 1, 3, 2, 2, 3) X(8, 1, 6, 2, 1, 3) X(8, 1, 1, 2, 2, 3) X(8, 1, 1, 2, 4, 3) X(8, 1, 2, 2, 1, 3) \
  X(4, 1, 3, 4, 1, 3) X(4, 1, 3, 4, 2, 3) \
  X(8, 1, 8, 2, 1, 4) X(8, 1, 8, 4, 1, 4) X(4, 1, 8, 4, 1, 4) X(2, 1, 8, 4, 1, 4) X(2, 1, 4, 4, 1, 4)

// fp8-weight instantiations (subset; KF even so one 16-B load carries two k-fragments; d = 3)
#define LSA_COOP_FP8_CONFIGS(X) \
  X(2, 1, 8, 4, 1, 3) X(4, 1, 8, 4, 1, 3) X(2, 1, 4, 4, 1, 3) X(4, 1, 4, 4, 1, 3) X(8, 1, 8, 4, 1, 3) X(8, 1, 4, 2, 1, 3) \
  X(2, 1, 8, 8, 1, 3) X(4, 1, 8, 8, 1, 3)

template <int EPI, bool FP8>
int dispatch(int mb, int tnw, int nw, int kf, int kw, int d, bool norm, const bf16_raw* x, int ldx, const int* a_rows,
             const bf16_raw* wp, int M, int N, int K, int SK, float eps, const EpiArgs& ep, float* slab, unsigned* cnt,
             const float* wscale, hipStream_t s) {
#define LSA_C(B, T, W, F, Q, DD)                                                                              \
  if (mb == B && tnw == T && nw == W && kf == F && kw == Q && d == DD)                                          \
    return launch<B, T, W, F, Q, DD, EPI, FP8>(norm, x, ldx, a_rows, wp, M, N, K, SK, eps, ep, slab, cnt, wscale, s);
  if constexpr (FP8) {
    LSA_COOP_FP8_CONFIGS(LSA_C)
  } else {
    LSA_COOP_CONFIGS(LSA_C)
  }
#undef LSA_C
  return LSA_UNSUPPORTED;
}

// K is split into 32*kf-k chunks, spread over the SK splits as evenly as possible.
// Workspace: slab >= SK*N*16*MB*4 + SK*(N/16/(nw*tnw))*16*MB*4 bytes (only when SK > 1);
// counters: N/16/(nw*tnw) zero-initialised uint32 (reset by the kernel itself).
template <bool FP8>
int coop_entry(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N, int K, int norm, float eps,
               int epi, const EpiArgs* ep, int tnw, int nw, int kf, int sk, int kw, int d, float* slab,
               unsigned* counters, const float* wscale, hipStream_t stream) {
  if (M < 1 || M > 128 || kf < 1 || K % (32 * kf) || ldx < K || sk < 0 || kw < 1) return LSA_BAD_SHAPE;
  if (kw > 1 && (K / (32 * kf)) % ((sk ? sk : 1) * kw)) return LSA_BAD_SHAPE;  // every k-group: same chunk count
  if (FP8 && (kf % 2 || !wscale)) return LSA_BAD_SHAPE;
  const int mb = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
  const int tg = nw * tnw;
  if (sk == 0) {  // ragged: tiles (SwiGLU: pairs) dealt to one workgroup per CU, at most tg each
    const int P = epi == EPI_SWIGLU ? 2 : 1, cu = n_cu();
    if (FP8 || epi == EPI_PARTIAL || N % (16 * P) || P % tnw) return LSA_BAD_SHAPE;
    const int units = N / 16 / P;
    if (units < cu || P * ((units + cu - 1) / cu) > tg) return LSA_BAD_SHAPE;
  } else if (N % (16 * tg) || sk > K / (32 * kf)) {
    return LSA_BAD_SHAPE;
  }
  if (epi == EPI_SWIGLU && tg % 2) return LSA_BAD_SHAPE;  // gate / up tile pairs stay in one workgroup
  if (sk > 1 && (!slab || !counters)) return LSA_BAD_SHAPE;
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
  const bool n = norm != 0;
#define LSA_D(E) dispatch<E, FP8>(mb, tnw, nw, kf, kw, d, n, xx, ldx, a_rows, w, M, N, K, sk, eps, *ep, slab, counters, wscale, stream)
  switch (epi) {
    case EPI_STORE: return LSA_D(EPI_STORE);
    case EPI_RESID: return LSA_D(EPI_RESID);
    case EPI_SWIGLU: return LSA_D(EPI_SWIGLU);
    case EPI_QKV: return LSA_D(EPI_QKV);
    case EPI_ARGMAX: return LSA_D(EPI_ARGMAX);
    case EPI_PARTIAL: return LSA_D(EPI_PARTIAL);
    default: return LSA_UNSUPPORTED;
  }
#undef LSA_D
}

}  // namespace

// K is split into 32*kf-k chunks, spread over the SK splits as evenly as possible; each split
// over kw k-groups of nw waves (kw > 1: (K/(32*kf)) % (sk*kw) == 0). EPI_PARTIAL: no in-kernel
// split reduction - split s stores its fp32 tile to ((float*)ep->out)[s][M][ldo] for
// lsa_resid_rmsnorm_partials. depth: register-ring depth of an instantiated config (3 or 4).
// Workspace: slab >= SK*N*16*MB*4 + SK*(N/16/(nw*tnw))*16*MB*4 bytes (only when SK > 1);
// counters: N/16/(nw*tnw) zero-initialised uint32 (reset by the kernel itself).
extern "C" int lsa_gemv_coop(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N, int K, int norm, float eps,
                             int epi, const EpiArgs* ep, int tnw, int nw, int kf, int sk, int kw, int depth, float* slab,
                             unsigned* counters, hipStream_t stream) {
  return coop_entry<false>(x, ldx, a_rows, wp, M, N, K, norm, eps, epi, ep, tnw, nw, kf, sk, kw, depth, slab, counters,
                           nullptr, stream);
}

#ifdef LSA_COOP_STAMPS
extern "C" int lsa_coop_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_coop_stamps), &buf, sizeof(buf)) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}
#endif

// Same with OCP fp8 e4m3 weights packed as in gemv_fp8.hip and fp32 per-row scales.
extern "C" int lsa_gemv_coop_fp8(const void* x, int ldx, const int* a_rows, const void* wq, const float* wscale, int M,
                                 int N, int K, int norm, float eps, int epi, const EpiArgs* ep, int tnw, int nw, int kf,
                                 int sk, float* slab, unsigned* counters, hipStream_t stream) {
  return coop_entry<true>(x, ldx, a_rows, wq, M, N, K, norm, eps, epi, ep, tnw, nw, kf, sk, 1, 3, slab, counters,
                          wscale, stream);
}
