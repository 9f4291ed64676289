// Projection GEMM with the weights streamed straight into MFMA B registers.
// hip.gemm routes it one round of 224-256 whole 128 x 192 tiles (the 7B qkv projection at
// 448-512 rows: 57.9 vs 68.1 us per layer in the headline decode step, profiles/r3_gemm_wr.md);
// gemm_sk.hip stays faster on every other measured shape.
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

// Diagnostic ablation builds only (-DLSA_WR_ABLATE=n into a separate .so, timed by
// scripts/gemm_wr_probe.py with WR_LIB=<that .so>; scripts/gpu_r3_wr_abl.sh; results are garbage): 1 = no VMEM in the loop, 2 = no barriers in the loop, 3 = no LDS reads in the
// loop, 4 = no MFMAs (faults: the unused asm load targets get reused), 5 = MFMAs only.
// The production library never defines it.
#ifndef LSA_WR_ABLATE
#define LSA_WR_ABLATE 0
#endif

template <int N>
LSA_DEVICE void wr_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

LSA_DEVICE void wr_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int FN, int NG = 1>
struct WrGeo {
  static constexpr int TN = FN * 16, BN = 4 * TN;
  static constexpr int NS = 4;                        // W register slots = A ring slots (distance 3)
  static constexpr int ADMA = WR_ABUF / 1024 / 4;     // A DMA instructions per wave per step (4)
  static constexpr int PER = 2 * FN + ADMA;           // VMEM instructions per wave per step
  static constexpr int ELD = TN + 4;                  // fp32 row stride of the epilogue image
  static constexpr int EPI_BYTES = NG * 4 * WR_BM * ELD * 4;  // NG = 2: group 1's partial image too
  static constexpr int RS_OFF = (NG * NS * WR_ABUF > EPI_BYTES ? NG * NS * WR_ABUF : EPI_BYTES);  // row rstd [128]
  static constexpr int SS_OFF = RS_OFF + WR_BM * 4;  // EPI_RESID + ss_out: 16-column sums of squares [128][BN / 16]
  static constexpr int SMEM = SS_OFF + WR_BM * (BN / 16) * 4;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(2 * PER <= 63, "vmcnt range");
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
// NG = 2 (experimental, scripts/gemm_wr_probe.py): two wave groups of 4 waves split every tile's
// K range in halves (two waves per SIMD, one from each group: while one waits, the other
// issues), each group with its own A ring; group 1 hands its partial accumulators to group 0
// through LDS before the epilogue. Both groups run the same number of steps, so every barrier
// pairs up.
template <int FN, int EPI, int NG>
LSA_DEVICE void gemm_wr_body(unsigned char* smem_all, const bf16_raw* __restrict__ A, int lda,
                             const bf16_raw* __restrict__ Wp, int M, int N, int K, const EpiArgs& ep, int MT,
                             int NT, int S) {
  using G_ = WrGeo<FN, NG>;
  constexpr int TN = G_::TN, BN = G_::BN, NS = G_::NS, ADMA = G_::ADMA, PER = G_::PER;
  const int lane = threadIdx.x & 63;
  const int wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wg >> 2, w = wg & 3;  // wave group, column owner within the group
  unsigned char* smem = smem_all + grp * (NS * WR_ABUF);  // this group's A ring
  const int G = gridDim.x;
  int g;
  {  // XCD-aware remap (bijective): blocks of one XCD get consecutive work ids
    const int hw = blockIdx.x, q = G / 8, r = G % 8, x = hw % 8;
    g = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + hw / 8;
  }
  const int n4 = K / (NS * WR_BK), KT32 = K >> 5;  // K in groups of NS 64-deep steps
  // A fragment read offsets inside one ring buffer (row lane%16 of a 16-row tile, 16-B chunk
  // kf*4 + lane/16 stored at chunk ^ (row % 8))
  const unsigned roff0 = (lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) * 16);
  const unsigned roff1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) * 16);

  // work item = (tile, K split sp): row tiles fastest, then column tiles, then splits (the items
  // running together share weight panels and K offsets); split sp covers the 64-deep steps
  // [k0, k1), both multiples of NS. S == 1 unless EPI_PARTIAL.
  for (int item = g; item < MT * NT * S; item += G) {
    const int tile = item % (MT * NT), sp = item / (MT * NT);
    const int mt = tile % MT, nt = tile / MT;
    int k0 = (sp * n4 / S) * NS, nsteps = ((sp + 1) * n4 / S) * NS;  // steps [k0, nsteps)
    if (NG == 2) {  // halves of the range, both multiples of NS (host: K % (2 NS 64) == 0)
      const int half = (nsteps - k0) / 2;
      k0 += grp * half;
      nsteps = k0 + half;
    }
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
      if constexpr (LSA_WR_ABLATE == 1 || LSA_WR_ABLATE == 5) if (ts > 2) return;
      const int j = v >> 1;
      const unsigned char* sb = wsb + (size_t)ts * 2048;
      if (v & 1)
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:1024" : "=v"(dst[j][1]) : "v"(wvo[j]), "s"(sb) : "memory");
      else
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst[j][0]) : "v"(wvo[j]), "s"(sb) : "memory");
    };
    // A DMA block s of step ts into ring slot `ring`
    auto aload = [&](int ring, int s, int ts) {
      if constexpr (LSA_WR_ABLATE == 1 || LSA_WR_ABLATE == 5) if (ts > 2) return;
      __builtin_amdgcn_global_load_lds(abase + (size_t)ts * (WR_BK * 2) + aoff[s],
                                       (__attribute__((address_space(3))) void*)(smem + ring * WR_ABUF + (w * ADMA + s) * 1024),
                                       16, 0, 0);
    };
    auto rd = [&](int slot, bool kf1, u32x4_t& dst, int i) {
      if constexpr (LSA_WR_ABLATE == 3 || LSA_WR_ABLATE == 5) { asm volatile("" : "+v"(dst)); return; }
      dst = ld16(smem + slot * WR_ABUF + i * 2048 + (kf1 ? roff1 : roff0));
    };
    // prologue: steps 0 .. NS-2 in flight (per step: W then A), A(0) kf0 frags read
    static_assert(NS == 4, "prologue issues steps 0, 1, 2");
#pragma unroll
    for (int v = 0; v < 2 * FN; ++v) wload(wr[0], v, k0);
#pragma unroll
    for (int s = 0; s < ADMA; ++s) aload(0, s, k0);
#pragma unroll
    for (int v = 0; v < 2 * FN; ++v) wload(wr[1], v, min(k0 + 1, nsteps - 1));
#pragma unroll
    for (int s = 0; s < ADMA; ++s) aload(1, s, min(k0 + 1, nsteps - 1));
#pragma unroll
    for (int v = 0; v < 2 * FN; ++v) wload(wr[2], v, min(k0 + 2, nsteps - 1));
#pragma unroll
    for (int s = 0; s < ADMA; ++s) aload(2, s, min(k0 + 2, nsteps - 1));
    wr_vm_wait<(NS - 2) * PER>();
    wr_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) rd(0, false, a0[i], i);

    // VMEM order per step: W(t+3) in phase A, A(t+3) in phase B; at barrier(t) A(t+1) and
    // W(t+1) must have landed: issued after them are W(t+2), A(t+2), W(t+3)
    constexpr int WAIT_MID = 2 * (2 * FN) + ADMA;
    auto step = [&](int t, auto slot_c) {
      constexpr int slot = decltype(slot_c)::value, nslot = (slot + NS - 1) % NS;
      const int tp = min(t + NS - 1, nsteps - 1);  // past the end: re-fetch the last step (dead)
      // phase A: row i's FN MFMAs of kf0, the kf1 frag read of row i, the weight prefetches
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = LSA_WR_ABLATE == 4 ? acc[i][j] : mfma16(a0[i], wr[slot][j][0], acc[i][j]);
        rd(slot, true, a1[i], i);
#pragma unroll
        for (int v = (i * 2 * FN) / 8; v < ((i + 1) * 2 * FN) / 8; ++v) wload(wr[nslot], v, tp);
        __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      wr_vm_wait<(LSA_WR_ABLATE == 1 || LSA_WR_ABLATE == 5 ? 0 : WAIT_MID)>();
      // barrier(t): every wave's share of A(t+1) is in LDS, and every wave has consumed its
      // reads of ring slot (t-1)%NS (they fed step t-1's MFMAs), which phase B refills
      if constexpr (LSA_WR_ABLATE != 2 && LSA_WR_ABLATE != 5) wr_barrier();
      // phase B: kf1 MFMAs, the reads of step t+1's kf0 frags, the A DMA of step t+3
      constexpr int s1 = (slot + 1) % NS;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = LSA_WR_ABLATE == 4 ? acc[i][j] : mfma16(a1[i], wr[slot][j][1], acc[i][j]);
        rd(s1, false, a0[i], i);
        if (i % 2 == 1) aload(nslot, i / 2, tp);
        __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    };
    for (int t = k0; t < nsteps; t += NS) {  // k0, nsteps multiples of NS
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
      step(t + 2, std::integral_constant<int, 2>{});
      step(t + 3, std::integral_constant<int, 3>{});
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

    if (NG == 2) {  // group 1's partial sums -> LDS -> added into group 0's accumulators
      float* part = reinterpret_cast<float*>(smem_all) + (4 + w) * (WR_BM * G_::ELD);
      if (grp == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[(i * 16 + 4 * (lane >> 4) + r) * G_::ELD + j * 16 + (lane & 15)] = acc[i][j][r];
      }
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] += part[(i * 16 + 4 * (lane >> 4) + r) * G_::ELD + j * 16 + (lane & 15)];
      }
    }
    // epilogue: fp32 tile through a wave-private LDS image; one lane per (row, 16 columns)
    // unit runs the row16 epilogues of epilogue.h (EPI_QKV: RoPE + KV-cache append; with
    // ss_in, the fused RMSNorm's row scale first, computed once per workgroup in gemm_sk's
    // summation order so both GEMMs produce the same bits)
    float* s_rs = reinterpret_cast<float*>(smem_all + G_::RS_OFF);
    if (EPI == EPI_QKV && ep.ss_in) {
      for (int r = threadIdx.x; r < WR_BM; r += WR_NTHR * NG) {
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
    float* img = reinterpret_cast<float*>(smem_all) + w * (WR_BM * G_::ELD);
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) img[(i * 16 + 4 * (lane >> 4) + r) * G_::ELD + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();  // the image and the row scales are complete
    const int col_base = nt * BN + w * TN;
    float* s_ss = reinterpret_cast<float*>(smem_all + G_::SS_OFF);
    constexpr int NU = (WR_BM * FN) / 64 / NG;  // unit passes per wave (NG = 2: the groups share each image)
#pragma unroll
    for (int s2 = 0; s2 < NU; ++s2) {
      const int u = lane + 64 * (grp * NU + s2), row = u / FN, j = u % FN;
      const int m = m0 + row;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4_t*>(v + 4 * q) = *reinterpret_cast<const f32x4_t*>(img + row * G_::ELD + j * 16 + 4 * q);
      if (EPI == EPI_RESID) {
        // residual add (+ bias); with ss_out, the sum of squares of the ROUNDED outputs of this
        // 16-column unit, combined per 64-column block below in lsa_row_ss's order
        float ssq = 0.f;
        if (m < M) {
          const int c0 = col_base + j * 16;
          epi_bias16(ep, c0, v);
          const bf16_raw* rr = ep.resid + (size_t)m * ep.ldr + c0;
          float x0[8], x1[8];
          unpack8(ld16(rr), x0);
          unpack8(ld16(rr + 8), x1);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            x0[q] += v[q];
            x1[q] += v[q + 8];
          }
          const u32x4_t p0 = pack8(x0), p1 = pack8(x1);
          bf16_raw* o = ep.out + (size_t)m * ep.ldo + c0;
          st16(o, p0);
          st16(o + 8, p1);
          unpack8(p0, x0);
          unpack8(p1, x1);
          ssq = ss16(x0, x1);
        }
        if (ep.ss_out) s_ss[row * (BN / 16) + w * FN + j] = ssq;
      } else if (m < M) {
        if (EPI == EPI_QKV && ep.ss_in) {
          const float rsc = s_rs[row];
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] *= rsc;
        }
        if (EPI == EPI_PARTIAL) {  // fp32 partial of split sp: ((float*)out)[sp][M][ldo]
          float* o = reinterpret_cast<float*>(ep.out) + ((size_t)sp * M + m) * ep.ldo + col_base + j * 16;
#pragma unroll
          for (int q = 0; q < 4; ++q) st16(o + 4 * q, __builtin_bit_cast(u32x4_t, *reinterpret_cast<const f32x4_t*>(v + 4 * q)));
        } else {
          epi_row16<EPI>(ep, m, col_base + j * 16, v);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (EPI == EPI_RESID && ep.ss_out) {  // per 64-column block: (s0 + s1) + (s2 + s3)
      __syncthreads();
      for (int r = threadIdx.x; r < WR_BM * (BN / 64); r += WR_NTHR * NG) {
        const int row = r / (BN / 64), b = r % (BN / 64);
        if (m0 + row < M) {
          const float* sq = s_ss + row * (BN / 16) + 4 * b;
          ep.ss_out[(size_t)(m0 + row) * ep.ss_n + ((nt * BN) >> 6) + b] =
              __fadd_rn(__fadd_rn(sq[0], sq[1]), __fadd_rn(sq[2], sq[3]));
        }
      }
    }
    wr_vm_wait<0>();  // this tile's stores retired: the next item's counted waits see only its own loads
    wr_barrier();     // the image is dead before the next tile's DMA reuses the LDS
  }
}

template <int FN, int EPI, int NG>
__global__ __launch_bounds__(WR_NTHR * NG) void gemm_wr_kernel(const bf16_raw* __restrict__ A, int lda,
                                                               const bf16_raw* __restrict__ Wp, int M, int N, int K,
                                                               EpiArgs ep, int MT, int NT, int S) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[WrGeo<FN, NG>::SMEM];
  gemm_wr_body<FN, EPI, NG>(smem, A, lda, Wp, M, N, K, ep, MT, NT, S);
}

template <int FN, int EPI, int NG = 1>
int wr_launch(const bf16_raw* A, int lda, const bf16_raw* W, int M, int N, int K, const EpiArgs& ep, int grid,
              int split, hipStream_t s) {
  constexpr int BN = WrGeo<FN, NG>::BN;
  const int MT = (M + WR_BM - 1) / WR_BM, NT = N / BN;
  const int items = MT * NT * split;
  gemm_wr_kernel<FN, EPI, NG><<<grid < items ? grid : items, WR_NTHR * NG, 0, s>>>(A, lda, W, M, N, K, ep, MT, NT,
                                                                                   split);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

}  // namespace

// 128-row x bn tiles, weights straight into MFMA registers (see the header comment). epi:
// EPI_STORE, EPI_RESID (out = resid + y; with ep->ss_out, the fused RMSNorm's per-64-column sums of
// squares of the rounded outputs, as gemm_sk), EPI_QKV (with the fused-RMSNorm row scale when
// ep->ss_in is set: K == 64 ss_n) or
// EPI_PARTIAL: every tile split into exactly `split` K ranges (multiples of 256), fp32 partial
// k to ((float*)ep->out)[k][M][ldo] (lsa_resid_rmsnorm_partials sums them); the caller checks
// the buffer holds split * M * ldo floats. bn: 128 / 192 / 256 with N % bn == 0; K % 256 == 0;
// grid: workgroups (work items beyond it loop). ng = 2 (experimental: two wave groups split
// each tile's K range; bn 128, EPI_STORE / EPI_RESID, split 1, K % 512 == 0). Returns LSA_BAD_SHAPE on any
// shape the kernel's indexing cannot take.
extern "C" int lsa_gemm_wr(const void* a, int lda, const void* wp, int M, int N, int K, int epi, const EpiArgs* ep,
                           int bn, int grid, int split, int ng, hipStream_t stream) {
  if (M < 1 || K < 4 * WR_BK || K % (4 * WR_BK) || lda < K || lda % 8 || grid < 1 || !ep) return LSA_BAD_SHAPE;
  if (bn != 128 && bn != 192 && bn != 256) return LSA_UNSUPPORTED;
  if (N % bn) return LSA_BAD_SHAPE;
  if (epi != EPI_STORE && epi != EPI_QKV && epi != EPI_PARTIAL && epi != EPI_RESID) return LSA_UNSUPPORTED;
  if (split < 1 || (split > 1 && epi != EPI_PARTIAL) || split > K / (4 * WR_BK)) return LSA_BAD_SHAPE;
  if (epi == EPI_PARTIAL && (!ep->out || ep->ldo < N || ep->ldo % 4)) return LSA_BAD_SHAPE;
  if (epi == EPI_STORE && (!ep->out || ep->ldo < N || ep->ldo % 8)) return LSA_BAD_SHAPE;
  if (epi == EPI_QKV && (!ep->k_cache || !ep->v_cache || !ep->slot || !ep->pos || !ep->out)) return LSA_BAD_SHAPE;
  if (epi == EPI_RESID && (!ep->out || !ep->resid || ep->ldo < N || ep->ldo % 8 || ep->ldr < N || ep->ldr % 8))
    return LSA_BAD_SHAPE;
  if (ep->ss_out && (epi != EPI_RESID || N % 64 || ep->ss_n != N / 64)) return LSA_BAD_SHAPE;
  if (ep->ss_in && (epi != EPI_QKV || ep->ss_n < 4 || ep->ss_n % 4 || K != 64 * ep->ss_n)) return LSA_BAD_SHAPE;
  if (ng != 1 && ng != 2) return LSA_UNSUPPORTED;
  const bf16_raw* A = static_cast<const bf16_raw*>(a);
  const bf16_raw* W = static_cast<const bf16_raw*>(wp);
  if (ng == 2) {
    if (bn != 128 || (epi != EPI_STORE && epi != EPI_RESID) || split != 1) return LSA_UNSUPPORTED;
    if (K % (8 * WR_BK)) return LSA_BAD_SHAPE;
    return epi == EPI_RESID ? wr_launch<2, EPI_RESID, 2>(A, lda, W, M, N, K, *ep, grid, 1, stream)
                            : wr_launch<2, EPI_STORE, 2>(A, lda, W, M, N, K, *ep, grid, 1, stream);
  }
#define LSA_WR(FN)                                                                                     \
  if (epi == EPI_RESID) return wr_launch<FN, EPI_RESID>(A, lda, W, M, N, K, *ep, grid, split, stream); \
  return epi == EPI_QKV     ? wr_launch<FN, EPI_QKV>(A, lda, W, M, N, K, *ep, grid, split, stream)     \
         : epi == EPI_PARTIAL ? wr_launch<FN, EPI_PARTIAL>(A, lda, W, M, N, K, *ep, grid, split, stream) \
                              : wr_launch<FN, EPI_STORE>(A, lda, W, M, N, K, *ep, grid, split, stream);
  if (bn == 128) { LSA_WR(2) }
  if (bn == 192) { LSA_WR(3) }
  LSA_WR(4)
#undef LSA_WR
}
