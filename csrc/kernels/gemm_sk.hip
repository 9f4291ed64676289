// Projection GEMM for > 128 rows (prompt prefill and big decode batches):
//   C[M, N] = A[M, K] @ W^T, bf16 in, fp32 accumulate, with the fused epilogues of epilogue.h
// (RoPE + KV-cache append | SwiGLU | residual add | store), replacing the reference's
// nn.Linear calls inside HF LlamaDecoderLayer (/root/reference/utils/shard_loader.py:66-74).
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", T1-T5):
//  * 256 x BN output tile (BN = 256 or 128) per 512-thread workgroup (8 waves, 2 per SIMD),
//    K step 64, one workgroup per CU, all LDS in ONE __shared__ array.
//  * Both operands reach LDS by LDS-DMA (global_load_lds_dwordx4): the packed-16x32 weights
//    (common.h) are already one lane-linear 1 KiB block per (16 cols, 32 k) fragment; the A
//    tile is fetched as whole 128-B rows (full cache lines: 5-12 % faster than gathering
//    fragment-order half lines, scripts/sk_ablate.py) into a row-major image whose 16-B chunks
//    are XOR-swizzled by row (per-lane source address), so every MFMA operand read is a
//    conflict-free ds_read_b128.
//  * Each K-tile runs as 4 phases (one output quadrant of 16 or 8 MFMAs each). The two wave
//    groups (waves 0-3 / 4-7, i.e. the two waves of every SIMD) run one raw s_barrier apart, so
//    one wave of a SIMD issues MFMAs while its partner issues LDS reads and DMA.
//  * The DMA for a buffer region is issued 5-6 phases ahead of its first read and retired by a
//    COUNTED s_waitcnt vmcnt (one K-tile of DMA stays in flight across every barrier).
//  * Work is split "data-parallel + stream-K": full rounds of 256-row x BN tiles go one per
//    workgroup (grouped tile order, XCD-aware block remap), the remaining tiles' K iterations
//    are spread evenly over the grid; a tile split between workgroups is combined by the last
//    arriving one (write-through fp32 slabs + an agent-scope ticket, §6 Guideline 16) which
//    then runs the fused epilogue.
//  * Epilogue: accumulators -> LDS (fp32) -> one thread per 16-column tile row -> the
//    vectorised row16 epilogues of epilogue.h (16-B stores).
#include "epilogue.h"

#include <type_traits>

namespace {

constexpr int BK = 64, NTHR = 512;

// BM x BN tile, BM = 256 or 128 (decode batches of <= 128 rows and M = 384 / 640 ...: no
// MFMA or A traffic on rows past M). BN = 256: 2 x 4 waves of BM/2 x 64; BN = 192 / 128: 4 x 2
// waves of BM/4 x 96 / BM/4 x 64.
// BN = 192 exists for shapes where 256-wide tiles leave CUs idle or need split-K fixups
// (Llama-2-7B qkv N=12288 at M=512: 2 x 64 = 128 tiles; gate_up N=22016: 230 tiles in one
// round at full K); N need not be a multiple of 192 (the last column tile is partial).
template <int BM, int BN, int NB>
struct Geo {
  static constexpr int WM = BN == 256 ? 2 : 4;   // wave grid
  static constexpr int WN = 8 / WM;
  static constexpr int TM = BM / WM, TN = BN / WN;  // per-wave output tile
  static constexpr int FM = TM / 16, FN = TN / 16;  // 16x16 MFMA tiles per wave
  static constexpr int AREG = (BM / 2) * BK * 2;    // bytes of one A region (16 / 8 KiB)
  static constexpr int BREG = (BN / 2) * BK * 2;    // bytes of one B region
  static constexpr int BUF = 2 * AREG + 2 * BREG;   // one K-tile
  static constexpr int AGL = AREG / 1024 / 8;       // DMA instructions per wave per A region
  static constexpr int BBLK = BREG / 1024;          // 1 KiB blocks per B region (16 / 12 / 8)
  // block b of a B region is issued by wave b % 8: with 12 blocks waves 0-3 issue 2 per
  // region and waves 4-7 one, so the per-wave counts (and counted waits) depend on the wave
  static constexpr int BGL = (BBLK + 7) / 8, BGL_LO = BBLK / 8, BHI_WAVES = BBLK % 8;
  static constexpr int NPT = 2 * AGL + 2 * BGL;     // DMA instructions per K-tile, waves < BHI_WAVES
  static constexpr int NPT_LO = 2 * AGL + 2 * BGL_LO;  // ... the other waves
  static constexpr int EROWS = (TN > 64 || TM < 64) ? 32 : 64;  // rows per epilogue transpose pass
  static constexpr int ELD = TN + 4;                // fp32 row stride of the transpose image
  static constexpr int EPI_BYTES = 8 * EROWS * ELD * 4;
  static constexpr int RS_OFF = (NB * BUF > EPI_BYTES ? NB * BUF : EPI_BYTES);  // row rstd of the tile [BM]
  static constexpr int SMEM = RS_OFF + BM * 4 + 16;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(BHI_WAVES == 0 || BGL_LO == 0 || BHI_WAVES == 4, "B blocks per wave");
  static_assert(AGL >= 1 && TM % EROWS == 0 && FM % 2 == 0, "tile geometry");
  static_assert(NB == 2 || BHI_WAVES == 0, "3-buffer ring needs the same DMA count in every wave");
};

struct SkParams {
  int M, N, K, lda;
  int MT, NT, NKT;       // BM-row tiles, BN-col tiles, 64-deep K tiles
  int G;                 // workgroups
  int dp_rounds;         // full rounds of whole tiles (tile r*G + g)
  int sk_tiles;          // tiles after the data-parallel rounds (the remainder)
  int split;             // 0: remainder spread by K iterations over the grid (stream-K);
                         // S >= 1: each remainder tile split into S equal K ranges (workgroup
                         // g < sk_tiles * S takes tile g % sk_tiles, range g / sk_tiles), so
                         // concurrently running workgroups stream the same K offsets (L2 reuse)
  int group_m;           // grouped tile order: this many row tiles share a column sweep
};

// Diagnostic ablation builds only (-DLSA_SK_ABLATE=n, scripts/sk_ablate.py; results are garbage,
// timings tell what bounds the main loop): 1 = no counted DMA waits in the loop, 2 = no DMA,
// 5 = A gathered as half-line fragment blocks (the pre-swizzle layout; reads then mismatch),
// 6 = no A DMA, 7 = no weight DMA, 8 = DMA only (no LDS reads, no MFMA), 9 = non-temporal
// weight DMA, 10 = no LDS reads (DMA + MFMA on stale registers), 11 = MFMA only,
// 3 = no MFMA, 4 = no barriers in the loop. The production library never defines it.
#ifndef LSA_SK_ABLATE
#define LSA_SK_ABLATE 0
#endif

// counted wait on the DMA queue (no other vector-memory op is in flight in the main loop)
template <int N>
LSA_DEVICE void vm_wait() {
  if constexpr (LSA_SK_ABLATE != 1 || N == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Diagnostic build only (-DLSA_GEMM_STAMPS, scripts/gemm_stamps.py): per-workgroup
// s_memrealtime stamps (100 MHz) at the phase boundaries of each work item, written by thread 0
// to a buffer nothing else reads. The production library never defines it.
#ifdef LSA_GEMM_STAMPS
__device__ unsigned long long* g_stamps;
#define LSA_STAMP(slot)                                                                        \
  do {                                                                                         \
    if (threadIdx.x == 0 && g_stamps) g_stamps[blockIdx.x * 32 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LSA_STAMP(slot) \
  do {                  \
  } while (0)
#endif

LSA_DEVICE void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

LSA_DEVICE void loop_barrier() {
  if constexpr (LSA_SK_ABLATE != 4) barrier();
}

LSA_DEVICE void glds16(const void* src, unsigned char* lds_base) {
  if constexpr (LSA_SK_ABLATE != 2 && LSA_SK_ABLATE != 11)
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
// weight stream: default cache policy (non-temporal weight DMA measured no better in the headline
// step, profiles/r3_gemm_nt_retune.jsonl; ablation build 9 keeps it for probes)
LSA_DEVICE void glds16_w(const void* src, unsigned char* lds_base) {
  if constexpr (LSA_SK_ABLATE == 9)
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 2 /* nt */);
  else
    glds16(src, lds_base);
}

// tile id -> (row tile, col tile): group_m row tiles sweep the column tiles together so the
// A panels and the weight panels of a round of 256 tiles both stay in L2 / the Infinity Cache
LSA_DEVICE void tile_coords(const SkParams& p, int tile, int& mt, int& nt) {
  const int per_group = p.group_m * p.NT;
  const int grp = tile / per_group, first = grp * p.group_m;
  const int gm = min(p.group_m, p.MT - first);
  const int r = tile - grp * per_group;
  mt = first + r % gm;
  nt = r / gm;
}

template <int BM, int BN, int EPI, int NB>
struct Kern {
  using G_ = Geo<BM, BN, NB>;
  static constexpr int WM = G_::WM, WN = G_::WN, TM = G_::TM, TN = G_::TN, FM = G_::FM, FN = G_::FN;
  static constexpr int AREG = G_::AREG, BREG = G_::BREG, BUF = G_::BUF, AGL = G_::AGL, BGL = G_::BGL,
                       NPT = G_::NPT, NPT_LO = G_::NPT_LO, BGL_LO = G_::BGL_LO, BHI_WAVES = G_::BHI_WAVES,
                       BBLK = G_::BBLK;
  static constexpr int HM = FM / 2, HN = FN / 2;  // quadrant size in 16x16 tiles

  unsigned char* smem;
  const bf16_raw* A;
  const bf16_raw* W;
  int tid, lane, w, wr, wc, group;
  const SkParams* p;

  // ---- DMA staging of one LDS region of local K-tile t ------------------------------------------
  // A region mh: the 128 rows wr'*TM + mh*TM/2 + i*16 + r16 (ordered (wr', i, r16)), 128 B each,
  // 16-B chunks XOR-swizzled by row%8; each DMA instruction fetches 8 whole rows (full lines)
  // Sources = wave-uniform segment base (SGPRs) + 32-bit per-lane offset (one VGPR per block
  // instead of a 64-bit pointer: the 256-wide tile needs every register it can keep).
  const unsigned char* a_seg;
  const unsigned char* b_seg;
  LSA_DEVICE void stage_a(int buf, int mh, const unsigned (&aoff)[2][AGL], int kt) {
    unsigned char* dst = smem + buf * BUF + mh * AREG;
    const unsigned char* base = a_seg + (size_t)kt * (BK * 2);
    if constexpr (LSA_SK_ABLATE == 6) return;
#pragma unroll
    for (int s = 0; s < AGL; ++s) glds16(base + aoff[mh][s], dst + (w * AGL + s) * 1024);
  }
  LSA_DEVICE void stage_b(int buf, int nh, const unsigned (&boff)[2][BGL], int kt) {
    unsigned char* dst = smem + buf * BUF + 2 * AREG + nh * BREG;
    const unsigned char* base = b_seg + (size_t)kt * 2048;
    if constexpr (LSA_SK_ABLATE == 7) return;
#pragma unroll
    for (int s = 0; s < BGL; ++s)
      if (s < BGL_LO || w < BHI_WAVES) glds16_w(base + boff[nh][s], dst + (s * 8 + w) * 1024);
  }
  // the same for a wave group known at compile time (HI: a wave w < BHI_WAVES, which issues
  // BGL B blocks per region; else BGL_LO): the main loop is instantiated per group, so neither
  // the DMA issue nor the counted waits branch on the wave id inside it
  template <bool HI>
  LSA_DEVICE void stage_b_g(int buf, int nh, const unsigned (&boff)[2][BGL], int kt) {
    unsigned char* dst = smem + buf * BUF + 2 * AREG + nh * BREG;
    const unsigned char* base = b_seg + (size_t)kt * 2048;
    if constexpr (LSA_SK_ABLATE == 7) return;
#pragma unroll
    for (int s = 0; s < BGL; ++s)
      if (s < BGL_LO || HI) glds16_w(base + boff[nh][s], dst + (s * 8 + w) * 1024);
  }
  template <bool HI>
  LSA_DEVICE void wait_tile_g() {
    vm_wait<(HI ? NPT : NPT_LO)>();
  }
  // counted wait keeping one K-tile of this wave's DMA in flight (+ EXTRA instructions)
  template <int EXTRA = 0>
  LSA_DEVICE void wait_tile() {
    if constexpr (NPT == NPT_LO) {
      vm_wait<NPT + EXTRA>();
    } else {
      if (w < BHI_WAVES) vm_wait<NPT + EXTRA>(); else vm_wait<NPT_LO + EXTRA>();
    }
  }
  // counted wait leaving one A and one B region of this wave's DMA in flight
  LSA_DEVICE void wait_ab() {
    if constexpr (NPT == NPT_LO) {
      vm_wait<AGL + BGL>();
    } else {
      if (w < BHI_WAVES) vm_wait<AGL + BGL>(); else vm_wait<AGL + BGL_LO>();
    }
  }

  // ---- one segment: K-tiles [ka, kb) of output tile (mt, nt), accumulated into acc -------------
  int stamp_base = 0;
  LSA_DEVICE void run_segment(f32x4_t (&acc)[FM][FN], int mt, int nt, int ka, int kb) {
    LSA_STAMP(stamp_base + 0);
    const SkParams& P = *p;
    const int n = kb - ka;
    const int m0 = mt * BM, n0 = nt * BN;
    const int KT32 = P.K >> 5;
    a_seg = reinterpret_cast<const unsigned char*>(A + (size_t)m0 * P.lda + ka * BK);
    b_seg = reinterpret_cast<const unsigned char*>(W) + ((size_t)(n0 >> 4) * KT32 + ka * 2) * 1024;
    unsigned aoff[2][AGL], boff[2][BGL];
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int s = 0; s < AGL; ++s) {
        // block b = 8 whole 128-B rows (full cache lines) of the region's row-major image, rows
        // ordered (wr', i, r16); lane -> row b*8 + lane/8, physical 16-B chunk lane%8 holding
        // logical chunk (lane%8) ^ (row%8) (XOR swizzle: conflict-free fragment reads in rd_a)
        const int b = w * AGL + s, wi = b >> 1, r16 = (b & 1) * 8 + (lane >> 3);
        const int wr_ = wi / HM, i = wi % HM, ch = (lane & 7) ^ ((lane >> 3) & 7);
        if constexpr (LSA_SK_ABLATE == 5) {  // (pre-swizzle fragment-order gather, half lines)
          const int row = min(m0 + wr_ * TM + mh * (TM / 2) + i * 16 + (lane & 15), P.M - 1) - m0;
          aoff[mh][s] = (unsigned)((row * P.lda + (b & 1) * 32 + 8 * (lane >> 4)) * 2);
          continue;
        }
        const int row = min(m0 + wr_ * TM + mh * (TM / 2) + i * 16 + r16, P.M - 1) - m0;
        aoff[mh][s] = (unsigned)((row * P.lda + ch * 8) * 2);
      }
    const int nt16_last = (P.N >> 4) - 1 - (n0 >> 4);  // partial last column tile (BN = 192): clamp
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int s = 0; s < BGL; ++s) {
        const int b = (s * 8 + w) % BBLK, kf = b & 1, wj = b >> 1;
        const int wc_ = wj / HN, j = wj % HN;
        const int ntl = min(wc_ * FN + nh * HN + j, nt16_last);
        boff[nh][s] = (unsigned)(((ntl * KT32 + kf) * 64 + lane) * 16);
      }

    // prologue. NB = 2: RA0(0) RB0(0) RB1(0) RA1(0) [RA0(1) RB0(1)];
    //           NB = 3: all four regions of tiles 0 [and 1]
    stage_a(0, 0, aoff, 0);
    stage_b(0, 0, boff, 0);
    stage_b(0, 1, boff, 0);
    stage_a(0, 1, aoff, 0);
    if (n > 1) {
      stage_a(1, 0, aoff, 1);
      stage_b(1, 0, boff, 1);
      if (NB == 3) {
        stage_b(1, 1, boff, 1);
        stage_a(1, 1, aoff, 1);
        vm_wait<BGL + AGL + NPT>();
      } else {
        wait_tile();
      }
    } else {
      wait_ab();
    }
    barrier();
    if (group) barrier();  // stagger: waves 4-7 run one barrier behind waves 0-3
    LSA_STAMP(stamp_base + 1);

    u32x4_t a[HM][2], b0[HN][2], b1[HN][2];
    // A fragment (row lane%16, k kf*32 + 8*(lane/16)) in the swizzled row-major image
    const unsigned roff0 = (lane & 15) * 128 + (((lane >> 4) ^ (lane & 7)) * 16);
    const unsigned roff1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ (lane & 7)) * 16);
    auto rd_a = [&](int buf, int mh) {
      if constexpr (LSA_SK_ABLATE == 8 || LSA_SK_ABLATE == 10 || LSA_SK_ABLATE == 11) return;
      const unsigned char* src = smem + buf * BUF + mh * AREG;
#pragma unroll
      for (int i = 0; i < HM; ++i) {
        a[i][0] = ld16(src + (wr * HM + i) * 2048 + roff0);
        a[i][1] = ld16(src + (wr * HM + i) * 2048 + roff1);
      }
    };
    auto rd_b = [&](int buf, int nh, u32x4_t (&bb)[HN][2]) {
      if constexpr (LSA_SK_ABLATE == 8 || LSA_SK_ABLATE == 10 || LSA_SK_ABLATE == 11) return;
      const unsigned char* src = smem + buf * BUF + 2 * AREG + nh * BREG + lane * 16;
#pragma unroll
      for (int j = 0; j < HN; ++j)
#pragma unroll
        for (int kf = 0; kf < 2; ++kf) bb[j][kf] = ld16(src + ((wc * HN + j) * 2 + kf) * 1024);
    };
    auto mma = [&](int mh, const u32x4_t (&bb)[HN][2], int nh) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (LSA_SK_ABLATE == 3 || LSA_SK_ABLATE == 8) {
#pragma unroll
        for (int kf = 0; kf < 2; ++kf) {
#pragma unroll
          for (int i = 0; i < HM; ++i) asm volatile("" ::"v"(a[i][kf]));
#pragma unroll
          for (int j = 0; j < HN; ++j) asm volatile("" ::"v"(bb[j][kf]));
        }
      } else {
#pragma unroll
        for (int kf = 0; kf < 2; ++kf)
#pragma unroll
          for (int i = 0; i < HM; ++i)
#pragma unroll
            for (int j = 0; j < HN; ++j)
              acc[mh * HM + i][nh * HN + j] = mfma16(a[i][kf], bb[j][kf], acc[mh * HM + i][nh * HN + j]);
      }
      __builtin_amdgcn_s_setprio(0);
    };

    // The main loop with every condition resolved at compile time: the K-tiles that stage both
    // later tiles (t + 2 < n), the one that stages only t + 1, and the last one are separate
    // instantiations of the same tile body (same stages, waits and barriers in the same order
    // as one loop with run-time tests - 18 branches and ~60 scalar instructions per K-tile
    // fewer, profiles/r5_gemm_pmc.md), and the body is instantiated per wave group
    const std::true_type T_{};
    const std::false_type F_{};
    auto main_loop = [&](auto hi_c) {
      constexpr bool HI = decltype(hi_c)::value;
      if constexpr (NB == 2) {
        // 2 buffers: RB1/RA1 of tile t+1 go into the other buffer, RA0/RB0 of tile t+2 into this
        // one right after their last reads; each region lands 5-6 phases after its DMA issue and
        // the counted wait keeps one K-tile of DMA in flight
        auto body = [&](int t, auto s1_c, auto s2_c) {
          constexpr bool S1 = decltype(s1_c)::value, S2 = decltype(s2_c)::value;
          const int cur = t & 1, nxt = cur ^ 1;
          rd_a(cur, 0);
          rd_b(cur, 0, b0);
          if constexpr (S1) { stage_b_g<HI>(nxt, 1, boff, t + 1); wait_tile_g<HI>(); } else vm_wait<0>();
          loop_barrier();
          mma(0, b0, 0);
          loop_barrier();
          rd_b(cur, 1, b1);
          if constexpr (S1) { stage_a(nxt, 1, aoff, t + 1); wait_tile_g<HI>(); } else vm_wait<0>();
          loop_barrier();
          mma(0, b1, 1);
          loop_barrier();
          rd_a(cur, 1);
          if constexpr (S2) { stage_a(cur, 0, aoff, t + 2); wait_tile_g<HI>(); } else vm_wait<0>();
          loop_barrier();
          mma(1, b1, 1);
          loop_barrier();
          if constexpr (S2) { stage_b_g<HI>(cur, 0, boff, t + 2); wait_tile_g<HI>(); } else vm_wait<0>();
          loop_barrier();
          mma(1, b0, 0);
          loop_barrier();
        };
        int t = 0;
        for (; t + 2 < n; ++t) body(t, T_, T_);
        if (t + 1 < n) {
          body(t, T_, F_);
          ++t;
        }
        body(t, F_, F_);
      } else {
        // 3 buffers: tile t+2 is staged during tile t into the buffer tile t-1 used, in read
        // order; the counted wait keeps the last 6 phases of DMA (~1.5 K-tiles) in flight
        int cur = 0, nx2 = 2;
        auto body = [&](int t, auto st_c) {
          constexpr bool ST = decltype(st_c)::value;
          rd_a(cur, 0);
          rd_b(cur, 0, b0);
          if constexpr (ST) { stage_a(nx2, 0, aoff, t + 2); vm_wait<NPT + 2 * AGL>(); } else vm_wait<0>();
          loop_barrier();
          mma(0, b0, 0);
          loop_barrier();
          rd_b(cur, 1, b1);
          if constexpr (ST) { stage_b_g<true>(nx2, 0, boff, t + 2); vm_wait<NPT + AGL + BGL>(); } else vm_wait<0>();
          loop_barrier();
          mma(0, b1, 1);
          loop_barrier();
          rd_a(cur, 1);
          if constexpr (ST) { stage_b_g<true>(nx2, 1, boff, t + 2); vm_wait<NPT + 2 * BGL>(); } else vm_wait<0>();
          loop_barrier();
          mma(1, b1, 1);
          loop_barrier();
          if constexpr (ST) { stage_a(nx2, 1, aoff, t + 2); vm_wait<NPT + AGL + BGL>(); } else vm_wait<0>();
          loop_barrier();
          mma(1, b0, 0);
          loop_barrier();
          cur = cur == 2 ? 0 : cur + 1;
          nx2 = nx2 == 2 ? 0 : nx2 + 1;
        };
        int t = 0;
        for (; t + 2 < n; ++t) body(t, T_);
        for (; t < n; ++t) body(t, F_);
      }
    };
    if constexpr (NPT == NPT_LO) {
      main_loop(T_);
    } else {
      if (w < BHI_WAVES) main_loop(T_); else main_loop(F_);
    }
    if (!group) barrier();  // re-align the two wave groups; every LDS read has retired
  }

  // ---- fp32 partial slab (fragment-native, write-through) ------------------------------------
  LSA_DEVICE void slab_store(float* slab, size_t slot, const f32x4_t (&acc)[FM][FN]) {
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(slab + slot * (size_t)(BM * BN), (short)0,
                                                                         BM * BN * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[i][j]), sr,
                                               ((w * FM * FN + i * FN + j) * 64 + lane) * 16, 0, 16);
  }
  // Adds partial slab ``slot`` into acc. The slab's fragment blocks (1 KiB, lane-linear) go
  // LDS-DMA -> this wave's private LDS ring (2 buffers of RP tile rows) -> registers, so RP*FN
  // write-through reads stay in flight while the previous group is added (the slab lines are
  // read sc1: they bypass this CU's L1, which may hold stale copies). Caller: every wave, LDS
  // free (and a barrier before the LDS is reused by other waves).
  LSA_DEVICE void slab_add(const float* slab, size_t slot, f32x4_t (&acc)[FM][FN]) {
    // RP tile rows (PB blocks) per pass, NP passes, DB ring buffers per wave: as much in flight
    // as this geometry's LDS allows (the ring must stay below the flag word at SMEM - 16)
    constexpr int AVAIL = G_::SMEM - 16;
    constexpr int RP = (FN <= 4 && FM % 2 == 0 && 8 * 2 * 2 * FN * 1024 <= AVAIL) ? 2 : 1;
    constexpr int NP = FM / RP, PB = RP * FN;
    constexpr int DB = (NP > 1 && 8 * 2 * PB * 1024 <= AVAIL) ? 2 : 1;
    static_assert(8 * DB * PB * 1024 <= AVAIL, "slab ring exceeds the LDS allocation");
    const unsigned char* src = reinterpret_cast<const unsigned char*>(slab + slot * (size_t)(BM * BN)) +
                               (size_t)(w * FM * FN) * 1024 + lane * 16;
    unsigned char* ring = smem + w * (DB * PB * 1024);
    auto issue = [&](int pass) {
#pragma unroll
      for (int q = 0; q < PB; ++q)
        __builtin_amdgcn_global_load_lds(src + ((pass * RP + q / FN) * FN + q % FN) * 1024,
                                         (__attribute__((address_space(3))) void*)(ring + ((pass % DB) * PB + q) * 1024),
                                         16, 0, 16 /* sc1 */);
    };
    issue(0);
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      if (DB == 2 && pass + 1 < NP) {
        issue(pass + 1);
        vm_wait<PB>();
      } else {
        vm_wait<0>();
      }
      const unsigned char* rb = ring + (pass % DB) * PB * 1024 + lane * 16;
#pragma unroll
      for (int q = 0; q < PB; ++q)
        acc[pass * RP + q / FN][q % FN] += __builtin_bit_cast(f32x4_t, ld16(rb + q * 1024));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads retired before the buffer is refilled
      __builtin_amdgcn_sched_barrier(0);
      if (DB == 1 && pass + 1 < NP) issue(pass + 1);
    }
  }

  // ---- fused epilogue through an LDS transpose -------------------------------------------------
  LSA_DEVICE void epilogue(const EpiArgs& ep, const f32x4_t (&acc)[FM][FN], int mt, int nt, int sp) {
    const SkParams& P = *p;
    constexpr int EROWS = G_::EROWS, ELD = G_::ELD, FPP = EROWS / 16;  // rows / fragments per pass
    float* img = reinterpret_cast<float*>(smem) + w * (EROWS * ELD);
    // fused RMSNorm: the rstd of each of the tile's BM rows from the producer's 64-column
    // partials, computed ONCE per workgroup (one thread per row, all of its partials' loads in
    // flight) and summed in the same order as before (bitwise-identical rstd). Before, every
    // wave column recomputed its rows' rstd per pass: 4x the partials traffic, +23 us on a
    // 2048-row gate_up (scripts/epi_cost_probe.py)
    float* s_rs = reinterpret_cast<float*>(smem + G_::RS_OFF);
    constexpr bool SS_IN = EPI == EPI_QKV || EPI == EPI_SWIGLU;
    if (SS_IN && ep.ss_in) {
      for (int r = tid; r < BM; r += NTHR) {
        const int m = min(mt * BM + r, P.M - 1);
        const float* sp = ep.ss_in + (size_t)m * ep.ss_n;
        float t = 0.f;
        for (int i0 = 0; i0 < ep.ss_n; i0 += 64) {
          f32x4_t q4[16];
#pragma unroll
          for (int j = 0; j < 16; ++j)
            q4[j] = i0 + 4 * j < ep.ss_n ? *reinterpret_cast<const f32x4_t*>(sp + i0 + 4 * j)
                                          : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (i0 + 4 * j < ep.ss_n) t += (q4[j][0] + q4[j][1]) + (q4[j][2] + q4[j][3]);
        }
        s_rs[r] = rsqrtf(t / (float)(64 * ep.ss_n) + ep.ss_eps);
      }
      __syncthreads();
    }
    constexpr int PASSES = TM / EROWS;
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const float* rs = s_rs + wr * TM + ps * EROWS;  // this pass's rows
#pragma unroll
      for (int i = 0; i < FPP; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            img[(i * 16 + 4 * (lane >> 4) + r) * ELD + j * 16 + (lane & 15)] = acc[ps * FPP + i][j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int row_base = mt * BM + wr * TM + ps * EROWS;
      const int col_base = nt * BN + wc * TN;
      if (EPI == EPI_SWIGLU) {
        // units: EROWS rows x FN/2 gate|up tile pairs
        constexpr int UNITS = EROWS * (FN / 2);
#pragma unroll
        for (int s = 0; s < (UNITS + 63) / 64; ++s) {
          const int u = lane + 64 * s, row = u / (FN / 2), pr = u % (FN / 2);
          const int m = (UNITS % 64 == 0 || u < UNITS) ? row_base + row : P.M;
          const float* src = img + row * ELD + pr * 32;
          float g[16], uu[16], v[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            *reinterpret_cast<f32x4_t*>(g + 4 * q) = *reinterpret_cast<const f32x4_t*>(src + 4 * q);
            *reinterpret_cast<f32x4_t*>(uu + 4 * q) = *reinterpret_cast<const f32x4_t*>(src + 16 + 4 * q);
          }
          const int c0 = col_base + pr * 32;
          if (m < P.M && (BN != 192 || c0 < P.N)) {
            if (ep.ss_in) {
              const float r = rs[row];
#pragma unroll
              for (int q = 0; q < 16; ++q) {
                g[q] *= r;
                uu[q] *= r;
              }
            }
            epi_bias16(ep, c0, g);
            epi_bias16(ep, c0 + 16, uu);
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = silu(g[q]) * uu[q];
            bf16_raw* o = ep.out + (size_t)m * ep.ldo + (c0 >> 1);
            st16(o, pack8(v));
            st16(o + 8, pack8(v + 8));
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < (EROWS * FN) / 64; ++s) {
          const int u = lane + 64 * s, row = u / FN, j = u % FN;
          const int m = row_base + row;
          const float* src = img + row * ELD + j * 16;
          float v[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4_t*>(v + 4 * q) = *reinterpret_cast<const f32x4_t*>(src + 4 * q);
          if (EPI == EPI_ARGMAX) {
            // largest key of the unit, then of the FN lanes of this row (consecutive lanes; FN
            // is a power of two for bn 128 / 256), one 64-bit atomic per row and wave
            const int c0 = col_base + j * 16;
            unsigned long long k = 0ull;
            if (m < P.M) {
              epi_bias16(ep, c0, v);
              k = argmax_key16(v, (unsigned)(c0 + ep.col_offset));
            }
#pragma unroll
            for (int o = 1; o < FN; o <<= 1) {
              const unsigned long long ko = __shfl_xor(k, o, 64);
              k = ko > k ? ko : k;
            }
            if (m < P.M && (lane % FN) == 0) atomicMax(&ep.keys[m], k);
          } else if (EPI == EPI_RESID && ep.ss_out) {
            // residual add + the row's sum of squares of the ROUNDED outputs over this wave's
            // 64 columns (FN = 4 consecutive lanes per row: bn 128 / 256), one float per block
            float ssq = 0.f;
            const int c0 = col_base + j * 16;
            if (m < P.M) {
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
            // (s0 + s1) + (s2 + s3) over the FN = 4 units of the 64-column block (lsa_row_ss order)
#pragma unroll
            for (int o = 1; o < FN; o <<= 1) ssq = __fadd_rn(ssq, __shfl_xor(ssq, o, 64));
            if (m < P.M && (lane % FN) == 0) ep.ss_out[(size_t)m * ep.ss_n + (col_base >> 6)] = ssq;
          } else if (m < P.M && (BN != 192 || col_base + j * 16 < P.N)) {
            if (EPI == EPI_QKV && ep.ss_in) {
              const float r = rs[row];
#pragma unroll
              for (int q = 0; q < 16; ++q) v[q] *= r;
            }
            if (EPI == EPI_PARTIAL) {  // fp32 partial of K range sp: 4 x 16-B stores
              float* o = reinterpret_cast<float*>(ep.out) + ((size_t)sp * P.M + m) * ep.ldo + col_base + j * 16;
#pragma unroll
              for (int q = 0; q < 4; ++q)
                st16(reinterpret_cast<bf16_raw*>(o + 4 * q), __builtin_bit_cast(u32x4_t, *reinterpret_cast<const f32x4_t*>(v + 4 * q)));
            } else {
              epi_row16<EPI>(ep, m, col_base + j * 16, v);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
};

template <int BM, int BN, int EPI, int NB>
__global__ __launch_bounds__(NTHR) void gemm_sk_kernel(const bf16_raw* __restrict__ A, const bf16_raw* __restrict__ W,
                                                        SkParams prm, EpiArgs ep, float* __restrict__ slab,
                                                        unsigned* __restrict__ counters) {
  using K_ = Kern<BM, BN, EPI, NB>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[Geo<BM, BN, NB>::SMEM];
  K_ k;
  k.smem = smem;
  k.A = A;
  k.W = W;
  k.p = &prm;
  k.tid = threadIdx.x;
  k.lane = threadIdx.x & 63;
  k.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  k.wr = k.w / K_::WN;
  k.wc = k.w % K_::WN;
  k.group = k.w >> 2;
  const int G = prm.G;
  // XCD-aware remap (bijective): blocks that share an XCD get consecutive work ids
  const int hw = blockIdx.x;
  int g;
  {
    const int q = G / 8, r = G % 8, x = hw % 8;
    g = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + hw / 8;
  }
  f32x4_t acc[K_::FM][K_::FN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < K_::FM; ++i)
#pragma unroll
      for (int j = 0; j < K_::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  };

  // One work loop (a single inlined copy of the segment and epilogue code keeps register
  // allocation within 256 VGPRs): first the data-parallel rounds (whole tiles r*G + g), then
  // this workgroup's stream-K iterations [lo, hi) of the remaining tiles' K loops.
  const long long S = (long long)prm.sk_tiles * prm.NKT;
  const long long lo = prm.sk_tiles ? (long long)g * S / G : 0, hi = prm.sk_tiles ? (long long)(g + 1) * S / G : 0;
  int* flag = reinterpret_cast<int*>(smem + Geo<BM, BN, NB>::SMEM - 16);
  int r = 0;
  long long it = lo;
  bool split_done = false;
  // split mode: U = sk_tiles * split work units spread EVENLY over the XCDs (units u, u+1 of
  // one K range - neighbouring tiles that share A or W panels - on one XCD); blocks beyond U idle
  int su = -1;
  if (prm.split) {
    const int U = prm.sk_tiles * prm.split, q = U / 8, rr = U % 8, x = hw % 8, j = hw / 8;
    if (j < (x < rr ? q + 1 : q)) su = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + j;
  }
  for (;;) {
    int tile, ts = 0, ka = 0, kb = prm.NKT, sp = 0;
    bool sk = false;
    if (r < prm.dp_rounds) {
      tile = r * G + g;
      ++r;
    } else if (prm.split) {
      if (split_done || su < 0) break;
      ts = su % prm.sk_tiles;
      sp = su / prm.sk_tiles;
      ka = sp * prm.NKT / prm.split;
      kb = (sp + 1) * prm.NKT / prm.split;
      tile = prm.dp_rounds * G + ts;
      split_done = true;
    } else if (it < hi) {
      ts = (int)(it / prm.NKT);
      ka = (int)(it - (long long)ts * prm.NKT);
      const long long tile_end = (long long)(ts + 1) * prm.NKT;
      kb = (int)((hi < tile_end ? hi : tile_end) - (long long)ts * prm.NKT);
      tile = prm.dp_rounds * G + ts;
      sk = true;
    } else {
      break;
    }
    const bool partial = ka != 0 || kb != prm.NKT;
    int mt, nt;
    tile_coords(prm, tile, mt, nt);
    zero();
    k.run_segment(acc, mt, nt, ka, kb);
    LSA_STAMP(k.stamp_base + 2);
    bool do_epi = true;
    if (partial && EPI != EPI_PARTIAL) {
      // contributors of this tile, in K order: split mode - workgroups ts + s * sk_tiles
      // (slot 0); stream-K - the workgroups whose iteration ranges intersect the tile's
      const long long t0 = (long long)ts * prm.NKT, t1 = t0 + prm.NKT;
      const int g_first = prm.split ? 0 : (int)(((t0 + 1) * G - 1) / S);
      const int g_last = prm.split ? prm.split - 1 : (int)((t1 * G - 1) / S);
      k.slab_store(slab, prm.split ? (size_t)su * 2 : (size_t)g * 2 + (it == lo ? 0 : 1), acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (k.tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(&counters[ts], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = old == (unsigned)(g_last - g_first);
      }
      __syncthreads();
      LSA_STAMP(k.stamp_base + 3);
      do_epi = *flag != 0;
      if (do_epi) {
        // fixed summation order (bitwise-reproducible results): with two contributors the
        // sum is commutative; with more, every partial - this one's too - is re-read in order
        const bool all = g_last - g_first > 1;
        if (all) zero();
        for (int ci = g_first; ci <= g_last; ++ci) {
          int c, slot;
          if (prm.split) {
            c = ts + ci * prm.sk_tiles;
            slot = 0;
          } else {
            c = ci;
            slot = (long long)c * S / G >= t0 ? 0 : 1;  // slot 0: c's range starts in this tile
          }
          if (c == (prm.split ? su : g) && !all) continue;
          k.slab_add(slab, (size_t)c * 2 + slot, acc);
        }
        if (k.tid == 0) __hip_atomic_store(&counters[ts], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // every wave's slab ring reads are done before the epilogue reuses LDS
      }
    }
    LSA_STAMP(k.stamp_base + 4);
    if (do_epi) k.epilogue(ep, acc, mt, nt, sp);
    LSA_STAMP(k.stamp_base + 5);
    k.stamp_base = k.stamp_base + 6 < 30 ? k.stamp_base + 6 : 24;
    __syncthreads();
    if (sk) it = (long long)ts * prm.NKT + kb;
  }
}

template <int BM, int BN, int EPI, int NB>
int launch(const bf16_raw* A, const bf16_raw* W, const SkParams& prm, const EpiArgs& ep, float* slab,
           unsigned* cnt, hipStream_t s) {
  gemm_sk_kernel<BM, BN, EPI, NB><<<prm.G, NTHR, 0, s>>>(A, W, prm, ep, slab, cnt);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

template <int BM, int EPI>
int dispatch(const bf16_raw* A, const bf16_raw* W, const SkParams& prm, const EpiArgs& ep, float* slab,
             unsigned* cnt, int bn, int nb, hipStream_t s) {
  if (bn == 256) {
    if constexpr (BM == 128) {
      if (nb == 3) return launch<BM, 256, EPI, 3>(A, W, prm, ep, slab, cnt, s);
    }
    return launch<BM, 256, EPI, 2>(A, W, prm, ep, slab, cnt, s);
  }
  if (bn == 192) return launch<BM, 192, EPI, 2>(A, W, prm, ep, slab, cnt, s);
  return nb == 3 ? launch<BM, 128, EPI, 3>(A, W, prm, ep, slab, cnt, s)
                 : launch<BM, 128, EPI, 2>(A, W, prm, ep, slab, cnt, s);
}

}  // namespace

// bm: tile height 256 or 128. bn: tile width 256 / 192 (192: N % 16 == 0, partial last tile) / 128.
// nb: DMA ring buffers, 2 or 3 (3 for bn 128, and bn 256 at bm 128; 0 = the default: 3 where
// allowed). grid: workgroups (<= 1024); dp: 1 = whole tiles in data-parallel rounds first (0 =
// all tiles are remainder).
// epi EPI_PARTIAL: every tile split into exactly `split` K ranges (tiles * split <= grid), fp32
// partial k stored to ((float*)ep->out)[k][M][ldo], no slabs or tickets (lsa_resid_rmsnorm_partials sums them).
// split: 0 = remainder by stream-K, S >= 1 = remainder tiles split into up to S K ranges
// (clamped to NKT and to grid / remainder tiles; stream-K when the remainder exceeds the grid).
// slab: >= 2 * grid * bm * bn floats and counters: >= remainder tiles (zeroed) when any tile is
// split. Returns LSA_BAD_SHAPE on any shape the kernel's indexing cannot take.
extern "C" int lsa_gemm_sk(const void* a, int lda, const void* wp, int M, int N, int K, int epi,
                           const EpiArgs* ep, int bm, int bn, int nb, int grid, int dp, int split, int group_m, float* slab,
                           unsigned* counters, long long slab_floats, int n_counters, hipStream_t stream) {
  if (M < 1 || K < BK || K % BK || lda < K || lda % 8 || !ep) return LSA_BAD_SHAPE;
  if (bn != 256 && bn != 192 && bn != 128) return LSA_UNSUPPORTED;
  if (bm != 256 && bm != 128) return LSA_UNSUPPORTED;
  const int BM = bm;
  if (nb == 0) nb = (bn == 128 || (bm == 128 && bn == 256)) ? 3 : 2;
  if (nb != 2 && !(nb == 3 && (bn == 128 || (bm == 128 && bn == 256)))) return LSA_UNSUPPORTED;
  if (bn == 192 ? (N % 16 || (epi == EPI_SWIGLU && N % 32)) : N % bn) return LSA_BAD_SHAPE;
  if (grid < 1 || grid > 1024 || group_m < 1) return LSA_BAD_SHAPE;
  if (epi == EPI_RESID && !ep->resid) return LSA_BAD_SHAPE;
  if (epi == EPI_QKV && (!ep->k_cache || !ep->v_cache || !ep->slot || !ep->pos)) return LSA_BAD_SHAPE;
  if (epi == EPI_ARGMAX ? (!ep->keys || bn == 192) : !ep->out) return LSA_BAD_SHAPE;
  if (ep->ss_out && (epi != EPI_RESID || bn == 192 || N % 64 || ep->ss_n != N / 64)) return LSA_BAD_SHAPE;
  if (ep->ss_in && ((epi != EPI_QKV && epi != EPI_SWIGLU) || ep->ss_n < 4 || ep->ss_n % 4 || K != 64 * ep->ss_n))
    return LSA_BAD_SHAPE;
  if (epi == EPI_PARTIAL && (split < 1 || ep->ldo < N || ep->ldo % 4)) return LSA_BAD_SHAPE;
  SkParams prm;
  prm.M = M;
  prm.N = N;
  prm.K = K;
  prm.lda = lda;
  prm.MT = (M + BM - 1) / BM;
  prm.NT = (N + bn - 1) / bn;
  prm.NKT = K / BK;
  prm.group_m = group_m;
  const long long tiles = (long long)prm.MT * prm.NT;
  if (tiles >= (1LL << 30)) return LSA_BAD_SHAPE;
  const long long iters = tiles * prm.NKT;
  prm.G = (int)(grid < iters ? grid : iters);
  prm.dp_rounds = dp ? (int)(tiles / prm.G) : 0;
  prm.sk_tiles = (int)(tiles - (long long)prm.dp_rounds * prm.G);
  prm.split = 0;
  if (epi == EPI_PARTIAL) {
    // every tile split into exactly `split` K ranges, one workgroup each, partial k written to
    // out[k]: the consumer sums exactly `split` partials, so nothing may be clamped here
    if (split > prm.NKT || tiles * split > grid) return LSA_BAD_SHAPE;
    prm.G = grid;
    prm.dp_rounds = 0;
    prm.sk_tiles = (int)tiles;
    prm.split = split;
  } else if (split > 0 && prm.sk_tiles > 0 && prm.sk_tiles <= prm.G) {
    // at most NKT ranges per tile and sk_tiles * split <= G workgroups
    prm.split = split < prm.NKT ? split : prm.NKT;
    if (prm.split > prm.G / prm.sk_tiles) prm.split = prm.G / prm.sk_tiles;
  } else if (prm.sk_tiles > 0 && (long long)prm.sk_tiles * prm.NKT < prm.G) {
    if (prm.dp_rounds > 0) {  // too few stream-K iterations for the grid: fold one round in
      prm.dp_rounds -= 1;
      prm.sk_tiles += prm.G;
    } else {
      prm.G = prm.sk_tiles * prm.NKT;  // every workgroup gets >= 1 iteration
    }
  }
  if (epi != EPI_PARTIAL && prm.sk_tiles > 0 &&
      (!slab || !counters || slab_floats < 2LL * prm.G * BM * bn || n_counters < prm.sk_tiles))
    return LSA_BAD_SHAPE;
  const bf16_raw* A = static_cast<const bf16_raw*>(a);
  const bf16_raw* W = static_cast<const bf16_raw*>(wp);
#define LSA_G(E) (bm == 256 ? dispatch<256, E>(A, W, prm, *ep, slab, counters, bn, nb, stream) \
                    : dispatch<128, E>(A, W, prm, *ep, slab, counters, bn, nb, stream))
  switch (epi) {
    case EPI_STORE: return LSA_G(EPI_STORE);
    case EPI_RESID: return LSA_G(EPI_RESID);
    case EPI_QKV: return LSA_G(EPI_QKV);
    case EPI_SWIGLU: return LSA_G(EPI_SWIGLU);
    case EPI_PARTIAL: return LSA_G(EPI_PARTIAL);
    case EPI_ARGMAX: return LSA_G(EPI_ARGMAX);
    default: return LSA_UNSUPPORTED;
  }
#undef LSA_G
}

#ifdef LSA_GEMM_STAMPS
extern "C" int lsa_gemm_sk_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}
#endif
