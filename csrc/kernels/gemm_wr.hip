// Projection GEMM with the weights streamed straight into MFMA B registers.
// hip.gemm routes to it from a measured per-shape table (ops/hip.py WR_ROUTES): the qkv and
// SwiGLU gate_up projections at the row counts where its 128-row tiles fill about one round
// (e.g. the 7B qkv at 448-512 rows: 57.9 vs 68.1 us per layer in the headline decode step,
// profiles/r3_gemm_wr.md; 3B / 13B shapes in profiles/r4_gemm_wr_shapes.jsonl and the engine
// A/B runs in profiles/r4_gemm_wr_engine_ab.txt). gemm_sk.hip keeps every other shape.
//
//   C[M, N] = A[M, K] @ W^T, bf16 in, fp32 accumulate.
//
// Why a second GEMM: gemm_sk stages BOTH operands through LDS (LDS-DMA) and runs 8 waves of
// 2 x 4 / 4 x 2 wave tiles; its ablation builds (profiles/r3_gemm_sk_ablation.jsonl) show the
// LDS traffic (DMA writes + fragment reads) costing about as much as the MFMAs at the 128 /
// 192-column tiles the decode shapes need. Here:
//  * 4 waves (one per SIMD), 128-row x BN tile, each wave owns ALL 128 rows x BN/4 columns, so
//    every weight fragment is used by exactly one wave: it is fetched with ONE
//    global_load_dwordx4 per lane (the packed-16x32 layout of common.h is already lane-linear
//    1 KiB per fragment) into registers, prefetched 3 K-steps ahead - no LDS for W at all.
//  * only A goes through LDS (LDS-DMA, whole 128-B rows, XOR-swizzled 16-B chunks as in
//    gemm_sk: conflict-free ds_read_b128 fragment reads), a 4-deep ring.
//  * LDS traffic per K-step: 16 KiB of DMA writes + 4 x 16 KiB of fragment reads, against
//    8 x FN x 2 MFMAs per wave: 37.5 % (BN 256) / 50 % (BN 192) of the MFMA time, where
//    gemm_sk's 256 x 128 tile is at ~87 %.
// Reference op: the nn.Linear calls of HF LlamaDecoderLayer (/root/reference/utils/shard_loader.py:66-74).
#include "epilogue.h"

#include <utility>

namespace {

constexpr int WR_BM = 128, WR_BK = 64, WR_NTHR = 256;
constexpr int WR_ABUF = WR_BM * WR_BK * 2;  // one A K-step image: 16 KiB

template <int N>
LSA_DEVICE void wr_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int... S, typename F>
LSA_DEVICE void wr_static_for(std::integer_sequence<int, S...>, F&& f) {
  (f(std::integral_constant<int, S>{}), ...);
}

LSA_DEVICE void wr_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int FN, int NS_>
struct WrGeo {
  static constexpr int TN = FN * 16, BN = 4 * TN;
  static constexpr int NS = NS_;                      // W register slots = A ring slots (distance NS-1)
  static constexpr int ADMA = WR_ABUF / 1024 / 4;     // A DMA instructions per wave per step (4)
  static constexpr int PER = 2 * FN + ADMA;           // VMEM instructions per wave per step
  static constexpr int ELD = TN + 4;                  // fp32 row stride of the epilogue image
  static constexpr int EPI_BYTES = 4 * WR_BM * ELD * 4;
  static constexpr int RS_OFF = (NS * WR_ABUF > EPI_BYTES ? NS * WR_ABUF : EPI_BYTES);  // row rstd [128]
  static constexpr int SMEM = RS_OFF + WR_BM * 4;
  // counted waits: the prologue leaves NS-2 steps in flight, the mid-step wait NS-3 steps + one
  // step's weights; vmcnt holds 6 bits
  static constexpr int WAIT_PRO = (NS - 2) * PER, WAIT_MID = (NS - 3) * PER + 2 * FN;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(NS >= 4 && WAIT_PRO <= 63 && WAIT_MID <= 63, "vmcnt range");
  static_assert(ADMA == 4, "one A DMA block per two rows of phase B");
};

// One output tile per iteration of a grid-stride loop; tiles ordered row-tile fastest so the
// MT row tiles sharing a weight panel run together (and on one XCD after the block remap).
// Pipeline of one 64-deep K-step t (two 32-deep MFMA fragments kf0 / kf1):
//   phase A: MFMAs of kf0 (A frags a0, read during step t-1) interleaved with the reads of
//            kf1's frags (a1) and the weight prefetch W(t+3) into register slot (t+3)%4 (2*FN
//            loads spread over the MFMAs - issued as one burst they stall the single wave on
//            the texture path)
//   vmcnt (W(t+2), A(t+2), W(t+3) may stay in flight) + barrier: A(t+1) is in LDS for every
//            wave, and every wave has consumed its reads of ring slot (t-1)%4
//   phase B: MFMAs of kf1 interleaved with the reads of step t+1's kf0 frags and the A DMA of
//            step t+3 into ring slot (t+3)%4 = (t-1)%4.
// (the body is a __device__ function: lambdas directly inside a __global__ template kept the
// host pass from emitting the kernel's launch stub)
template <int FN, int NS_, int EPI>
LSA_DEVICE void gemm_wr_body(unsigned char* smem, const bf16_raw* __restrict__ A, int lda,
                             const bf16_raw* __restrict__ Wp, int M, int N, int K, const EpiArgs& ep, int MT,
                             int NT) {
  using G_ = WrGeo<FN, NS_>;
  constexpr int TN = G_::TN, BN = G_::BN, NS = G_::NS, ADMA = G_::ADMA;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // column owner
  const int G = gridDim.x;
  int g;
  {  // XCD-aware remap (bijective): blocks of one XCD get consecutive work ids
    const int hw = blockIdx.x, q = G / 8, r = G % 8, x = hw % 8;
    g = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + hw / 8;
  }
  const int KT32 = K >> 5;
  // A fragment read offsets inside one ring buffer (row lane%16 of a 16-row tile, 16-B chunk
  // kf*4 + lane/16 stored at chunk ^ (row % 8))
  const unsigned roff0 = (lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) * 16);
  const unsigned roff1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) * 16);

  // work item = tile: row tiles fastest, then column tiles (the items running together share
  // weight panels); every tile covers the whole K range (64-deep steps [0, nsteps), K % 64 == 0)
  for (int tile = g; tile < MT * NT; tile += G) {
    const int mt = tile % MT, nt = tile / MT;
    const int k0 = 0, nsteps = K / WR_BK;
    const int m0 = mt * WR_BM, n16 = (nt * BN + w * TN) >> 4;  // this wave's first 16-col tile
    // A DMA: wave w fills blocks w*ADMA + s (8 rows x 128 B each) of every ring buffer
    unsigned aoff[ADMA];
#pragma unroll
    for (int s = 0; s < ADMA; ++s) {
      const int row = (w * ADMA + s) * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((lane >> 3) & 7);
      aoff[s] = (unsigned)((min(m0 + row, M - 1) * lda + ch * 8) * 2);
    }
    const unsigned char* abase = reinterpret_cast<const unsigned char*>(A);
    // weights: wave-uniform base of this wave's column panel (SGPRs; + 2 KiB per K-step) and a
    // per-lane offset per 16-column tile j (lane * 16 + j * KT32 KiB): the loads use the saddr
    // form, no per-load 64-bit address VALU (the single wave is issue-bound, profiles/r3_gemm_wr.md)
    const unsigned char* wsb = reinterpret_cast<const unsigned char*>(Wp) + (size_t)n16 * KT32 * 1024;
    unsigned wvo[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) wvo[j] = (unsigned)(lane * 16 + j * KT32 * 1024);

    f32x4_t acc[8][FN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    u32x4_t wr[NS][FN][2];  // indexed by compile-time slots only (the loop is unrolled by NS)
    u32x4_t a0[8], a1[8];

    // Weight fragment v = (j, kf) of step ts into register slot SLOT. Inline asm: the compiler
    // cannot count a register load whose value is used NS-1 steps later and would drain the
    // whole prefetch (vmcnt(0)) before the first MFMA of every step; the counted wait in the
    // step covers these loads.
    auto wload = [&](u32x4_t (&dst)[FN][2], int v, int ts) {
      const int j = v >> 1;
      const unsigned char* sb = wsb + (size_t)ts * 2048;
      if (v & 1)
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:1024" : "=v"(dst[j][1]) : "v"(wvo[j]), "s"(sb) : "memory");
      else
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst[j][0]) : "v"(wvo[j]), "s"(sb) : "memory");
    };
    // A DMA block s of step ts into ring slot `ring`
    auto aload = [&](int ring, int s, int ts) {
      __builtin_amdgcn_global_load_lds(abase + (size_t)ts * (WR_BK * 2) + aoff[s],
                                       (__attribute__((address_space(3))) void*)(smem + ring * WR_ABUF + (w * ADMA + s) * 1024),
                                       16, 0, 0);
    };
    auto rd = [&](int slot, bool kf1, u32x4_t& dst, int i) {
      dst = ld16(smem + slot * WR_ABUF + i * 2048 + (kf1 ? roff1 : roff0));
    };
    // prologue: steps 0 .. NS-2 in flight (per step: W then A), A(0) kf0 frags read
    wr_static_for(std::make_integer_sequence<int, NS - 1>{}, [&](auto sc) {
      constexpr int S = decltype(sc)::value;
#pragma unroll
      for (int v = 0; v < 2 * FN; ++v) wload(wr[S], v, min(k0 + S, nsteps - 1));
#pragma unroll
      for (int s = 0; s < ADMA; ++s) aload(S, s, min(k0 + S, nsteps - 1));
    });
    wr_vm_wait<G_::WAIT_PRO>();
    wr_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) rd(0, false, a0[i], i);

    // VMEM order per step: W(t+NS-1) in phase A, A(t+NS-1) in phase B; at barrier(t) A(t+1)
    // and W(t+1) must have landed: issued after them are W/A(t+2 .. t+NS-2) and W(t+NS-1)
    constexpr int WAIT_MID = G_::WAIT_MID;
    auto step = [&](int t, auto slot_c) {
      constexpr int slot = decltype(slot_c)::value, nslot = (slot + NS - 1) % NS;
      const int tp = min(t + NS - 1, nsteps - 1);  // past the end: re-fetch the last step (dead)
      // phase A: row i's FN MFMAs of kf0, the kf1 frag read of row i, the weight prefetches
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a0[i], wr[slot][j][0], acc[i][j]);
        rd(slot, true, a1[i], i);
#pragma unroll
        for (int v = (i * 2 * FN) / 8; v < ((i + 1) * 2 * FN) / 8; ++v) wload(wr[nslot], v, tp);
        __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      wr_vm_wait<WAIT_MID>();
      // barrier(t): every wave's share of A(t+1) is in LDS, and every wave has consumed its
      // reads of ring slot (t-1)%NS (they fed step t-1's MFMAs), which phase B refills
      wr_barrier();
      // phase B: kf1 MFMAs, the reads of step t+1's kf0 frags, the A DMA of step t+3
      constexpr int s1 = (slot + 1) % NS;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a1[i], wr[slot][j][1], acc[i][j]);
        rd(s1, false, a0[i], i);
        if (i % 2 == 1) aload(nslot, i / 2, tp);
        __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    };
    for (int t = k0; t < nsteps; t += NS) {  // k0 a multiple of NS; a partial last group is cut short
      wr_static_for(std::make_integer_sequence<int, NS>{}, [&](auto sc) {
        if (t + decltype(sc)::value < nsteps) step(t + decltype(sc)::value, sc);
      });
    }
    wr_vm_wait<0>();  // the dead prefetches land before the LDS is reused
    // ... and before their destination registers are: the compiler sees the last group's weight
    // prefetches as dead values and could hand their registers to epilogue values while the
    // loads are still in flight - keeping them live up to here (after the wait) rules that out
#pragma unroll
    for (int sl = 0; sl < NS; ++sl)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(wr[sl][j][0]), "v"(wr[sl][j][1]));
    wr_barrier();

    // epilogue: fp32 tile through a wave-private LDS image; one lane per (row, 16 columns)
    // unit runs the row16 epilogues of epilogue.h (EPI_QKV: RoPE + KV-cache append), or per
    // (row, gate/up tile pair) the SwiGLU; with ss_in, the fused RMSNorm's row scale first,
    // computed once per workgroup in gemm_sk's summation order so both GEMMs produce the same bits
    constexpr bool NORM_IN = EPI == EPI_QKV || EPI == EPI_SWIGLU;
    float* s_rs = reinterpret_cast<float*>(smem + G_::RS_OFF);
    if (NORM_IN && ep.ss_in) {
      for (int r = threadIdx.x; r < WR_BM; r += WR_NTHR) {
        const int m = min(m0 + r, M - 1);
        const float* sp = ep.ss_in + (size_t)m * ep.ss_n;
        float tsum = 0.f;
        for (int i0 = 0; i0 < ep.ss_n; i0 += 64) {
          f32x4_t q4[16];
#pragma unroll
          for (int j = 0; j < 16; ++j)
            q4[j] = i0 + 4 * j < ep.ss_n ? *reinterpret_cast<const f32x4_t*>(sp + i0 + 4 * j)
                                          : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (i0 + 4 * j < ep.ss_n) tsum += (q4[j][0] + q4[j][1]) + (q4[j][2] + q4[j][3]);
        }
        s_rs[r] = rsqrtf(tsum / (float)(64 * ep.ss_n) + ep.ss_eps);
      }
    }
    float* img = reinterpret_cast<float*>(smem) + w * (WR_BM * G_::ELD);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) img[(i * 16 + 4 * (lane >> 4) + r) * G_::ELD + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();  // the image and the row scales are complete
    const int col_base = nt * BN + w * TN;
    if constexpr (EPI == EPI_SWIGLU) {
      // 16-column tiles interleave gate / up (packing.fuse_gate_up): this wave's FN tiles are
      // FN / 2 (gate, up) pairs; pair p of the wave writes output columns col_base / 2 + 16 p
      constexpr int FP = FN / 2, NUP = (WR_BM * FP) / 64;
      static_assert(FN % 2 == 0, "SwiGLU needs whole gate / up tile pairs per wave");
#pragma unroll
      for (int s2 = 0; s2 < NUP; ++s2) {
        const int u = lane + 64 * s2, row = u / FP, jp = u % FP;
        const int m = m0 + row;
        float g[16], up[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          *reinterpret_cast<f32x4_t*>(g + 4 * q) = *reinterpret_cast<const f32x4_t*>(img + row * G_::ELD + (2 * jp) * 16 + 4 * q);
          *reinterpret_cast<f32x4_t*>(up + 4 * q) =
              *reinterpret_cast<const f32x4_t*>(img + row * G_::ELD + (2 * jp + 1) * 16 + 4 * q);
        }
        if (m < M) {
          const float rsc = ep.ss_in ? s_rs[row] : 1.f;
#pragma unroll
          for (int q = 0; q < 16; ++q) g[q] = silu(g[q] * rsc) * (up[q] * rsc);
          bf16_raw* o = ep.out + (size_t)m * ep.ldo + col_base / 2 + jp * 16;
          st16(o, pack8(g));
          st16(o + 8, pack8(g + 8));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      wr_vm_wait<0>();
      wr_barrier();
      continue;
    }
    constexpr int NU = (WR_BM * FN) / 64;  // unit passes per wave
#pragma unroll
    for (int s2 = 0; s2 < NU; ++s2) {
      const int u = lane + 64 * s2, row = u / FN, j = u % FN;
      const int m = m0 + row;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4_t*>(v + 4 * q) = *reinterpret_cast<const f32x4_t*>(img + row * G_::ELD + j * 16 + 4 * q);
      if (m < M) {
        if (EPI == EPI_QKV && ep.ss_in) {
          const float rsc = s_rs[row];
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] *= rsc;
        }
        epi_row16<EPI>(ep, m, col_base + j * 16, v);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    wr_vm_wait<0>();  // this tile's stores retired: the next item's counted waits see only its own loads
    wr_barrier();     // the image is dead before the next tile's DMA reuses the LDS
  }
}

template <int FN, int NS, int EPI>
__global__ __launch_bounds__(WR_NTHR) void gemm_wr_kernel(const bf16_raw* __restrict__ A, int lda,
                                                          const bf16_raw* __restrict__ Wp, int M, int N, int K,
                                                          EpiArgs ep, int MT, int NT) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[WrGeo<FN, NS>::SMEM];
  gemm_wr_body<FN, NS, EPI>(smem, A, lda, Wp, M, N, K, ep, MT, NT);
}

template <int FN, int NS, int EPI>
int wr_launch(const bf16_raw* A, int lda, const bf16_raw* W, int M, int N, int K, const EpiArgs& ep, int grid,
              hipStream_t s) {
  constexpr int BN = WrGeo<FN, NS>::BN;
  const int MT = (M + WR_BM - 1) / WR_BM, NT = N / BN;
  const int items = MT * NT;
  gemm_wr_kernel<FN, NS, EPI><<<grid < items ? grid : items, WR_NTHR, 0, s>>>(A, lda, W, M, N, K, ep, MT, NT);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

}  // namespace

// 128-row x bn tiles, weights straight into MFMA registers (see the header comment). epi:
// EPI_STORE, EPI_QKV or EPI_SWIGLU (bn 128 / 256; gate / up tiles interleaved), the last two with
// the fused-RMSNorm row scale when ep->ss_in is set (K == 64 ss_n).
// bn: 128 / 192 / 256 with N % bn == 0; K % 64 == 0; grid: workgroups (tiles beyond it loop).
// Returns LSA_BAD_SHAPE on any shape the kernel's indexing cannot take.
// (Ring depth: 4 slots. 6 and 8 slots - weights prefetched 5 / 7 K-steps ahead - measured no
// faster on any 7B projection shape, profiles/r4_gemm_wr_depth.jsonl: the weight stream is not
// latency-bound.)
extern "C" int lsa_gemm_wr(const void* a, int lda, const void* wp, int M, int N, int K, int epi, const EpiArgs* ep,
                           int bn, int grid, hipStream_t stream) {
  if (M < 1 || K < WR_BK || K % WR_BK || lda < K || lda % 8 || grid < 1 || !ep) return LSA_BAD_SHAPE;
  if (bn != 128 && bn != 192 && bn != 256) return LSA_UNSUPPORTED;
  if (N % bn) return LSA_BAD_SHAPE;
  if (epi != EPI_STORE && epi != EPI_QKV && epi != EPI_SWIGLU) return LSA_UNSUPPORTED;
  if (epi == EPI_SWIGLU && bn == 192) return LSA_UNSUPPORTED;  // 3 tiles per wave: no whole gate/up pairs
  if (epi == EPI_STORE && (!ep->out || ep->ldo < N || ep->ldo % 8)) return LSA_BAD_SHAPE;
  if (epi == EPI_SWIGLU && (!ep->out || ep->ldo < N / 2 || ep->ldo % 8 || ep->act || ep->bias)) return LSA_BAD_SHAPE;
  if (epi == EPI_QKV && (!ep->k_cache || !ep->v_cache || !ep->slot || !ep->pos || !ep->out)) return LSA_BAD_SHAPE;
  if (ep->ss_out) return LSA_BAD_SHAPE;
  if (ep->ss_in && (epi == EPI_STORE || ep->ss_n < 4 || ep->ss_n % 4 || K != 64 * ep->ss_n)) return LSA_BAD_SHAPE;
  const bf16_raw* A = static_cast<const bf16_raw*>(a);
  const bf16_raw* W = static_cast<const bf16_raw*>(wp);
#define LSA_WR(FN)                                                                                    \
  return epi == EPI_QKV ? wr_launch<FN, 4, EPI_QKV>(A, lda, W, M, N, K, *ep, grid, stream)         \
                        : wr_launch<FN, 4, EPI_STORE>(A, lda, W, M, N, K, *ep, grid, stream);
  if (epi == EPI_SWIGLU)
    return bn == 128 ? wr_launch<2, 4, EPI_SWIGLU>(A, lda, W, M, N, K, *ep, grid, stream)
                     : wr_launch<4, 4, EPI_SWIGLU>(A, lda, W, M, N, K, *ep, grid, stream);
  if (bn == 128) { LSA_WR(2) }
  if (bn == 192) { LSA_WR(3) }
  LSA_WR(4)
#undef LSA_WR
}
