// Prefill projection GEMM: C[M, N] = A[M, K] @ W^T for M > 16 (prompt tokens), bf16 in,
// fp32 accumulate, with the fused epilogues of epilogue.h.
//
// Tile 128 (rows) x 64*TN (cols) x 64 (k) per 4-wave workgroup. The A tile is staged
// global -> VGPR -> LDS (XOR-swizzled 16-byte chunks, double-buffered, one barrier per
// K-tile; loads for tile t+2 are issued before the MFMAs of tile t, cdna_hip_programming.md
// §5.5 T14). The B operand needs no LDS at all: the packed-16x32 weight layout (common.h)
// gives every wave its MFMA B fragments as contiguous 1 KiB loads, prefetched two K-tiles
// ahead in registers. Each wave owns TN 16-column tiles x all 128 rows (8 x TN
// v_mfma_f32_16x16x32_bf16 accumulators).
//
// The reference runs these as separate nn.Linear calls inside HF LlamaDecoderLayer
// (/root/reference/utils/shard_loader.py:66-74); here RoPE+KV append, SwiGLU and residual
// adds run in the epilogue.
#include "epilogue.h"

namespace {

constexpr int BM = 128, BK = 64, GWAVES = 4, GTHR = GWAVES * LSA_WAVE;

LSA_DEVICE int lds_off(int row, int chunk) {  // byte offset of 16-B chunk in the A tile
  // 128-B rows: two rows share a 256-B bank line, so XOR with (row >> 1) & 7 makes the 16
  // rows of one ds_read_b128 pass hit all 64 banks (row & 7 was 2-way conflicted)
  return row * (BK * 2) + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int TN, int EPI>
__global__ __launch_bounds__(GTHR) void gemm_packed_kernel(const bf16_raw* __restrict__ A, int lda,
                                                           const bf16_raw* __restrict__ wp, int M,
                                                           int N, int K, EpiArgs ep, int SK,
                                                           float* __restrict__ slab,
                                                           unsigned* __restrict__ counters) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BM * BK * 2];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int MT = (M + BM - 1) / BM;
  const int NTILE = MT * (N / (16 * GWAVES * TN));
  const int tile = blockIdx.x % NTILE, split = blockIdx.x / NTILE;
  const int mt = tile % MT, ct = tile / MT;
  const int m0 = mt * BM;
  const int KT = K >> 5;          // 32-wide k fragments
  const int NKT_ALL = K / BK;     // 64-wide k tiles; split s owns [kt_lo, kt_hi)
  const int kt_lo = split * NKT_ALL / SK, kt_hi = (split + 1) * NKT_ALL / SK;
  const int NKT = kt_hi - kt_lo;
  const int ntile0 = ct * (GWAVES * TN) + w * TN;  // this wave's first 16-col tile

  // A staging: 1024 chunks of 16 B per tile, 4 per thread. Rows past M load row M-1 (valid
  // memory) and are zeroed at LDS-store time, so the loads stay unconditional.
  // Buffer loads with a wave-uniform SGPR offset per K-tile (no 64-bit address temporaries for
  // the compiler to rematerialise / merge across the unrolled steps).
  struct AV { u32x4_t v[4]; };
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0x7fffffff, 0x00020000);
  int a_voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + GTHR * i, row = c >> 3, ch = c & 7;
    a_voff[i] = (min(m0 + row, M - 1) * lda + ch * 8) * 2;
  }
  const int b_tile0 = __builtin_amdgcn_readfirstlane(ntile0);
  auto load_a = [&](int t) -> AV {
    AV a;
#pragma unroll
    for (int i = 0; i < 4; ++i) a.v[i] = __builtin_amdgcn_raw_buffer_load_b128(ar, a_voff[i], (kt_lo + t) * BK * 2, 0);
    return a;
  };
  auto store_a = [&](int buf, const AV& a) {
    unsigned char* base = smem + buf * (BM * BK * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + GTHR * i, row = c >> 3, ch = c & 7;
      st16(base + lds_off(row, ch), m0 + row < M ? a.v[i] : u32x4_t{0u, 0u, 0u, 0u});
    }
  };
  auto load_b = [&](u32x4_t (&b)[2][TN], int t) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        b[ks][tn] = __builtin_amdgcn_raw_buffer_load_b128(br, lane * 16, ((b_tile0 + tn) * KT + (kt_lo + t) * 2 + ks) * 1024, 0);
  };

  f32x4_t acc[BM / 16][TN];
#pragma unroll
  for (int rb = 0; rb < BM / 16; ++rb)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[rb][tn] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int cur, const u32x4_t (&b)[2][TN]) {
    const unsigned char* base = smem + cur * (BM * BK * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int rb = 0; rb < BM / 16; ++rb) {
        const int row = rb * 16 + (lane & 15);
        const u32x4_t a = *reinterpret_cast<const u32x4_t*>(base + lds_off(row, ks * 4 + (lane >> 4)));
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[rb][tn] = mfma16(a, b[ks][tn], acc[rb][tn]);
      }
    }
  };

  // Prefetch distance 2 K-tiles for both operands (3-deep register rings): at ~1-2 us of
  // memory latency and ~0.2-0.4 us of MFMA work per K-tile, one tile of look-ahead left the
  // small-M grids (M 129..1024: few workgroups, 64 K-tiles each) latency-bound. A(t+1) is
  // issued before B(t+1) so waiting for it (LDS store) never drains the B prefetch (vmcnt
  // is in order); tail indices are clamped so every wait is a static count.
  {
    u32x4_t bX[2][TN], bY[2][TN], bZ[2][TN];
    AV aX, aY, aZ;
    const int last = NKT - 1;
    auto clampt = [&](int t) { return t < last ? t : last; };
    aX = load_a(0);
    load_b(bX, 0);
    aY = load_a(clampt(1));
    load_b(bY, clampt(1));
    store_a(0, aX);
    __syncthreads();
    auto step = [&](int t, u32x4_t (&bc)[2][TN], u32x4_t (&b2)[2][TN], AV& a1, AV& a2) {
      a2 = load_a(clampt(t + 2));
      load_b(b2, clampt(t + 2));
      __builtin_amdgcn_sched_barrier(0);
      compute(t & 1, bc);
      __builtin_amdgcn_sched_barrier(0);
      store_a((t + 1) & 1, a1);
      __syncthreads();
    };
    for (int t = 0;;) {
      step(t, bX, bZ, aY, aZ);
      if (++t > last) break;
      step(t, bY, bX, aZ, aX);
      if (++t > last) break;
      step(t, bZ, bY, aX, aY);
      if (++t > last) break;
    }
  }

  if (SK > 1) {
    // Split-K hand-off, sc1 form (as in gemv_coop.hip): fragment-native fp32 partials, one
    // 16-B write-through store per accumulator; the last-arriving split reads every partial
    // back into the same register layout (fixed split order -> deterministic) and runs the
    // fused epilogue below.
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slab, (short)0, 0x7fffffff, 0x00020000);
    constexpr int PER_WAVE = (BM / 16) * TN * 64 * 4;  // floats
    const int my_base = (tile * GWAVES + w) * PER_WAVE * 4;  // bytes within one split
    const int split_bytes = NTILE * GWAVES * PER_WAVE * 4;
#pragma unroll
    for (int rb = 0; rb < BM / 16; ++rb)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[rb][tn]), sr,
                                               my_base + ((rb * TN + tn) * 64 + lane) * 16, split * split_bytes, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(&counters[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)(SK - 1);
    }
    __syncthreads();
    if (!s_last) return;
#pragma unroll
    for (int rb = 0; rb < BM / 16; ++rb)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) acc[rb][tn] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < SK; ++q) {
      f32x4_t v[BM / 16][TN];
#pragma unroll
      for (int rb = 0; rb < BM / 16; ++rb)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          v[rb][tn] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                      sr, my_base + ((rb * TN + tn) * 64 + lane) * 16, q * split_bytes, 16));
#pragma unroll
      for (int rb = 0; rb < BM / 16; ++rb)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[rb][tn] += v[rb][tn];
    }
    if (tid == 0) __hip_atomic_store(&counters[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // epilogue: acc[rb][tn][r] = C[m0 + rb*16 + (lane>>4)*4 + r][(ntile0+tn)*16 + (lane&15)]
  const int n = lane & 15;
#pragma unroll
  for (int rb = 0; rb < BM / 16; ++rb) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gm = m0 + rb * 16 + (lane >> 4) * 4 + r;
      if (EPI == EPI_SWIGLU) {
        const float g = acc[rb][0][r], u = acc[rb][1][r];
        if (gm < M) ep.out[(size_t)gm * ep.ldo + (ntile0 / 2) * 16 + n] = f2bf(silu(g) * u);
      } else {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const float v = acc[rb][tn][r];
          const int col = (ntile0 + tn) * 16 + n;
          if (EPI == EPI_QKV) {
            const float vp = __shfl_xor(v, 8, 64);
            if (gm < M)
              epi_qkv_store(ep, gm, col, v + epi_bias(ep, col), vp + epi_bias(ep, col ^ 8), ep.pos[gm], ep.slot[gm]);
          } else if (gm < M) {
            if (EPI == EPI_STORE)
              ep.out[(size_t)gm * ep.ldo + col] = f2bf(epi_act(ep, v + epi_bias(ep, col)));
            else if (EPI == EPI_RESID)
              ep.out[(size_t)gm * ep.ldo + col] = f2bf(bf2f(ep.resid[(size_t)gm * ep.ldr + col]) + v + epi_bias(ep, col));
          }
        }
      }
    }
  }
}

template <int TN, int EPI>
int launch(const bf16_raw* A, int lda, const bf16_raw* wp, int M, int N, int K, const EpiArgs& ep, int sk,
           float* slab, unsigned* cnt, hipStream_t s) {
  const int MT = (M + BM - 1) / BM, CT = N / (16 * GWAVES * TN);
  gemm_packed_kernel<TN, EPI><<<MT * CT * sk, GTHR, 0, s>>>(A, lda, wp, M, N, K, ep, sk, slab, cnt);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

}  // namespace

extern "C" int lsa_gemm(const void* a, int lda, const void* wp, int M, int N, int K, int epi,
                        const EpiArgs* ep, int tn, int sk, float* slab, unsigned* counters, hipStream_t stream) {
  if (M < 1 || K % BK || lda < K || sk < 1 || sk > K / BK) return LSA_BAD_SHAPE;
  // 32-bit buffer offsets: both operands (and the split-K slab) must stay below 2 GiB
  if ((long long)M * lda * 2 >= 0x7fffffffLL || (long long)N * K * 2 >= 0x7fffffffLL) return LSA_BAD_SHAPE;
  if (tn != 1 && tn != 2) return LSA_UNSUPPORTED;
  if (N % (16 * GWAVES * tn)) return LSA_BAD_SHAPE;
  if (sk > 1) {
    const long long mpad = (long long)((M + BM - 1) / BM) * BM;
    if (!slab || !counters || sk * mpad * N * 4 >= 0x7fffffffLL) return LSA_BAD_SHAPE;
  }
  const bf16_raw* A = static_cast<const bf16_raw*>(a);
  const bf16_raw* W = static_cast<const bf16_raw*>(wp);
#define LSA_G(T, E) launch<T, E>(A, lda, W, M, N, K, *ep, sk, slab, counters, stream)
  switch (epi) {
    case EPI_STORE: return tn == 2 ? LSA_G(2, EPI_STORE) : LSA_G(1, EPI_STORE);
    case EPI_RESID: return tn == 2 ? LSA_G(2, EPI_RESID) : LSA_G(1, EPI_RESID);
    case EPI_QKV: return tn == 2 ? LSA_G(2, EPI_QKV) : LSA_G(1, EPI_QKV);
    case EPI_SWIGLU:
      if (tn != 2) return LSA_BAD_SHAPE;
      return LSA_G(2, EPI_SWIGLU);
    default: return LSA_UNSUPPORTED;
  }
#undef LSA_G
}
