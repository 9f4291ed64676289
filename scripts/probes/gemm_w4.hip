// Projection GEMM, one wave per SIMD with large per-wave tiles (a main loop
// built differently from gemm_sk's, not a control-flow edit of it).
//
//   C[M, N] = A[M, K] @ W^T, bf16 in, fp32 accumulate, W in the packed-16x32 layout (common.h).
//
// Why: gemm_sk runs 8 waves (two per SIMD) of 128 x 64 / 64 x 96 wave tiles with 8 raw barriers
// per 64-deep K-tile; its counters (profiles/r5_gemm_pmc.md) show waves parked 36-56 % of their
// cycles at barriers / waits. hipBLASLt's kernels at these shapes pair one wave per SIMD with big
// wave tiles (profiles/r4_hipblaslt_kernels.md). Here:
//  * 256 threads = 4 waves, one per SIMD; a 256 x 256 output tile, each wave 128 x 128 (8 x 8
//    16x16 MFMA tiles: 256 accumulator registers, which the compiler keeps in AGPRs - the kernel
//    runs at one wave per SIMD and may use all 512 registers);
//  * 32-deep K stages in a 4-slot LDS ring (4 x 32 KiB), both operands by LDS-DMA
//    (global_load_lds_dwordx4) straight into MFMA fragment order, so every fragment read is one
//    lane-linear, conflict-free ds_read_b128: the packed weights are already 1 KiB fragments,
//    A is gathered fragment-wise (16 rows x 64 B per DMA instruction);
//  * ONE raw s_barrier per stage (64 MFMAs per wave = 1,024 MFMA cycles per SIMD): the stage's
//    MFMAs are interleaved with the reads of the NEXT stage's fragments (double-buffered
//    registers) and the DMA of the stage three ahead; a counted vmcnt keeps one stage of DMA in
//    flight across every barrier (cdna_hip_programming.md §5 'Pipelining across barriers').
// Ring invariants at the top of stage s: the fragments of s are in registers (reads issued during
// s-1), stage s+1 has landed and is visible (vmcnt + barrier at the end of s-1), the DMA of s+2
// is in flight. Slot (s+3)%4 = (s-1)%4 is free: its fragments were read during s-2 and retired
// (lgkmcnt(0)) before the barrier that ended s-2.
// Reference op: the nn.Linear calls of HF LlamaDecoderLayer (/root/reference/utils/shard_loader.py:66-74).
#include "../../csrc/kernels/epilogue.h"

namespace {

constexpr int W4_BM = 256, W4_BN = 256, W4_BK = 32, W4_NTHR = 256, W4_NS = 4;
constexpr int W4_STAGE = (W4_BM + W4_BN) * W4_BK * 2;  // 32 KiB: 16 A fragments + 16 W fragments
constexpr int W4_SMEM = W4_NS * W4_STAGE;              // 128 KiB
constexpr int W4_GM = 16;                                // row tiles per group (tile order)

LSA_DEVICE void w4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
LSA_DEVICE void w4_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

LSA_DEVICE void w4_glds(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

struct W4Frags {
  u32x4_t a[8], b[8];
};

// Reads the wave's 16 fragments of one stage from ring slot `slot`.
LSA_DEVICE void w4_read(W4Frags& f, const unsigned char* slot, int wr, int wc, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f.a[i] = ld16(slot + (wr * 8 + i) * 1024 + lane * 16);
#pragma unroll
  for (int j = 0; j < 8; ++j) f.b[j] = ld16(slot + (16 + wc * 8 + j) * 1024 + lane * 16);
}

// One stage: the 64 MFMAs of `cur`, interleaved with the reads of `nxt` from `nslot` and (when
// DMA) the wave's 8 DMA pieces of stage t into `dslot`. V (schedule variant, A/B only):
// 0 = one DMA piece every 8 MFMAs, order pinned by sched_barrier; 1 = all 8 DMA pieces issued
// before the MFMAs; 2 = no pinning, sched_group_barrier hints (4 MFMA, 1 DS read[, 1 VMEM]).
template <bool DMA, int V>
LSA_DEVICE void w4_stage(f32x4_t (&acc)[8][8], const W4Frags& cur, W4Frags& nxt, const unsigned char* nslot,
                         unsigned char* dslot, const unsigned char* asrc, const unsigned char* bsrc,
                         const unsigned (&aoff)[4], const unsigned (&boff)[4], int w, int wr, int wc, int lane) {
  auto piece = [&](int p) {
    if (p < 4)
      w4_glds(asrc + aoff[p], dslot + (w * 4 + p) * 1024);
    else
      w4_glds(bsrc + boff[p - 4], dslot + (16 + w * 4 + p - 4) * 1024);
  };
  if (DMA && V == 1) {
#pragma unroll
    for (int p = 0; p < 8; ++p) piece(p);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = q >> 1, j0 = (q & 1) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j0 + j] = mfma16(cur.a[i], cur.b[j0 + j], acc[i][j0 + j]);
    if (q < 8)
      nxt.a[q] = ld16(nslot + (wr * 8 + q) * 1024 + lane * 16);
    else
      nxt.b[q - 8] = ld16(nslot + (16 + wc * 8 + (q - 8)) * 1024 + lane * 16);
    if (DMA && V != 1 && (q & 1)) piece(q >> 1);
    if (V == 2) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
      if (DMA && (q & 1)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 VMEM read
    } else {
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Stage s: MFMAs of `cur` + reads of stage s+1 into `nxt` (+ the DMA of stage s+3 when DMA),
// then the counted wait and the stage's one barrier.
template <bool DMA, int V>
LSA_DEVICE void w4_step(f32x4_t (&acc)[8][8], const W4Frags& cur, W4Frags& nxt, unsigned char* smem, int s,
                        const unsigned char* asrc, const unsigned char* bsrc, const unsigned (&aoff)[4],
                        const unsigned (&boff)[4], int w, int wr, int wc, int lane) {
  const unsigned char* nslot = smem + ((s + 1) % W4_NS) * W4_STAGE;
  w4_stage<DMA, V>(acc, cur, nxt, nslot, smem + ((s + 3) % W4_NS) * W4_STAGE, asrc, bsrc, aoff, boff, w, wr, wc, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (DMA)
    w4_vm_wait<8>();  // stage s+2 landed (s+3 stays in flight)
  else
    w4_vm_wait<0>();
  w4_barrier();
}

template <int EPI, int V>
__global__ __launch_bounds__(W4_NTHR, 1) void gemm_w4_kernel(const bf16_raw* __restrict__ A, int lda,
                                                           const bf16_raw* __restrict__ Wp, int M, int N, int K,
                                                           EpiArgs ep, int MT, int NT) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[W4_SMEM];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int G = gridDim.x;
  int g;
  {  // XCD-aware remap (bijective): blocks of one XCD get consecutive work ids
    const int hw = blockIdx.x, q = G / 8, r = G % 8, x = hw % 8;
    g = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + hw / 8;
  }
  const int KT32 = K >> 5, nst = KT32;
  const unsigned char* Ab = reinterpret_cast<const unsigned char*>(A);
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(Wp);

  for (int tile = g; tile < MT * NT; tile += G) {
    // grouped order: W4_GM row tiles sweep all column tiles together, so one round of 256 tiles
    // touches W4_GM A panels and every W panel (at M = 16,384: 32 + 32 MB, Infinity-Cache
    // resident) instead of every A panel (128 MB, re-streamed from HBM once per column round)
    int mt, nt;
    {
      const int per = W4_GM * NT, grp = tile / per, first = grp * W4_GM;
      const int gm = min(W4_GM, MT - first), r = tile - grp * per;
      mt = first + r % gm;
      nt = r / gm;
    }
    const int m0 = mt * W4_BM, n0 = nt * W4_BN;
    // DMA sources: A fragment w*4+p = rows m0 + (w*4+p)*16 + lane%16, 16-B chunk lane/16 of the
    // stage's 64 B; W fragment w*4+p = 16-col tile n0/16 + w*4 + p, the stage's 1 KiB block
    unsigned aoff[4], boff[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = min(m0 + (w * 4 + p) * 16 + (lane & 15), M - 1);
      aoff[p] = (unsigned)((row * lda + 8 * (lane >> 4)) * 2);
      const int n16 = min((n0 >> 4) + w * 4 + p, (N >> 4) - 1);
      boff[p] = (unsigned)(((size_t)n16 * KT32 * 64 + lane) * 16);
    }
    auto a_at = [&](int s) { return Ab + (size_t)s * (W4_BK * 2); };
    auto b_at = [&](int s) { return Wb + (size_t)s * 1024; };
    auto issue = [&](int s) {
      unsigned char* d = smem + (s % W4_NS) * W4_STAGE;
#pragma unroll
      for (int p = 0; p < 4; ++p) w4_glds(a_at(s) + aoff[p], d + (w * 4 + p) * 1024);
#pragma unroll
      for (int p = 0; p < 4; ++p) w4_glds(b_at(s) + boff[p], d + (16 + w * 4 + p) * 1024);
    };

    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // prologue: stages 0..2 in flight, 0 and 1 landed and visible, fragments of 0 read
    issue(0);
    issue(min(1, nst - 1));
    issue(min(2, nst - 1));
    w4_vm_wait<8>();
    w4_barrier();
    W4Frags X, Y;
    w4_read(X, smem, wr, wc, lane);

    // every stage issues one stage of DMA, 3 ahead; past the last stage it re-fetches the last
    // stage into the free slot (2-3 wasted stages per tile, < 3 % at K = 4,096) so that ONE loop
    // body with one counted wait covers the whole K range - a separate tail with its own waits
    // made the compiler spill the accumulators. K % 64 == 0: an even number of stages.
    for (int s = 0; s < nst; s += 2) {
      w4_step<true, V>(acc, X, Y, smem, s, a_at(min(s + 3, nst - 1)), b_at(min(s + 3, nst - 1)), aoff, boff, w, wr, wc,
                    lane);
      w4_step<true, V>(acc, Y, X, smem, s + 1, a_at(min(s + 4, nst - 1)), b_at(min(s + 4, nst - 1)), aoff, boff, w, wr,
                    wc, lane);
    }
    w4_vm_wait<0>();  // the re-fetches have landed before the next tile restages slots 0-2
    w4_barrier();                // every wave is done with the ring before the next tile restages it

    // epilogue: C rows m0 + wr*128 + i*16 + 4*(lane/16) + r, cols n0 + wc*128 + j*16 + lane%16;
    // buffer stores (rows >= M fall outside the resource and are dropped: no branch, so the
    // accumulator indices stay static)
    const __amdgpu_buffer_rsrc_t orc =
        __builtin_amdgcn_make_buffer_rsrc(ep.out, (short)0, (int)min((long long)M * ep.ldo * 2, 0x7fffffffLL), 0x00020000);
    const int rb = m0 + wr * 128 + 4 * (lane >> 4), cb = n0 + wc * 128 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          __builtin_amdgcn_raw_buffer_store_b16(f2bf(acc[i][j][r]), orc, ((rb + i * 16 + r) * ep.ldo + cb + j * 16) * 2, 0,
                                                0);
  }
}

}  // namespace

// Plain-store GEMM (EPI_STORE) on the one-wave-per-SIMD 256 x 256 kernel. N % 256 == 0,
// K % 64 == 0; grid 0 = min(tiles, 256).
extern "C" int lsa_gemm_w4(const void* a, int lda, const void* wp, int M, int N, int K, const EpiArgs* ep, int grid,
                           int variant, hipStream_t stream) {
  if (M < 1 || K < 2 * W4_BK || K % (2 * W4_BK) || N % W4_BN || lda < K || lda % 8 || !ep || !ep->out) return LSA_BAD_SHAPE;
  const int MT = (M + W4_BM - 1) / W4_BM, NT = N / W4_BN;
  const long long tiles = (long long)MT * NT;
  if (grid <= 0) grid = tiles < 256 ? (int)tiles : 256;
  const bf16_raw* A = static_cast<const bf16_raw*>(a);
  const bf16_raw* W = static_cast<const bf16_raw*>(wp);
  if (variant == 1)
    gemm_w4_kernel<EPI_STORE, 1><<<grid, W4_NTHR, 0, stream>>>(A, lda, W, M, N, K, *ep, MT, NT);
  else if (variant == 2)
    gemm_w4_kernel<EPI_STORE, 2><<<grid, W4_NTHR, 0, stream>>>(A, lda, W, M, N, K, *ep, MT, NT);
  else
    gemm_w4_kernel<EPI_STORE, 0><<<grid, W4_NTHR, 0, stream>>>(A, lda, W, M, N, K, *ep, MT, NT);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}
