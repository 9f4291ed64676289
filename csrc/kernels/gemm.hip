// Prefill projection GEMM: C[M, N] = A[M, K] @ W^T for M > 16 (prompt tokens), bf16 in,
// fp32 accumulate, with the fused epilogues of epilogue.h.
//
// Tile 128 (rows) x 64*TN (cols) x 64 (k) per 4-wave workgroup. The A tile is staged
// global -> VGPR -> LDS (XOR-swizzled 16-byte chunks, double-buffered, one barrier per
// K-tile; loads for tile t+1 are issued before the MFMAs of tile t, cdna_hip_programming.md
// §5.5 T14). The B operand needs no LDS at all: the packed-16x32 weight layout (common.h)
// gives every wave its MFMA B fragments as contiguous 1 KiB loads, prefetched one K-tile
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
  return row * (BK * 2) + ((chunk ^ (row & 7)) << 4);
}

template <int TN, int EPI>
__global__ __launch_bounds__(GTHR) void gemm_packed_kernel(const bf16_raw* __restrict__ A, int lda,
                                                           const bf16_raw* __restrict__ wp, int M,
                                                           int N, int K, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BM * BK * 2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int MT = (M + BM - 1) / BM;
  const int mt = blockIdx.x % MT, ct = blockIdx.x / MT;
  const int m0 = mt * BM;
  const int KT = K >> 5;          // 32-wide k fragments
  const int NKT = K / BK;         // 64-wide k tiles
  const int ntile0 = ct * (GWAVES * TN) + w * TN;  // this wave's first 16-col tile

  // A staging: 1024 chunks of 16 B per tile, 4 per thread
  u32x4_t areg[4];
  auto load_a = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + GTHR * i, row = c >> 3, ch = c & 7;
      const int gm = m0 + row;
      areg[i] = gm < M ? ld16(A + (size_t)gm * lda + t * BK + ch * 8) : u32x4_t{0u, 0u, 0u, 0u};
    }
  };
  auto store_a = [&](int buf) {
    unsigned char* base = smem + buf * (BM * BK * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + GTHR * i, row = c >> 3, ch = c & 7;
      st16(base + lds_off(row, ch), areg[i]);
    }
  };
  u32x4_t bcur[2][TN], bnext[2][TN];
  auto load_b = [&](u32x4_t (&b)[2][TN], int t) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        b[ks][tn] = ld16(wp + ((size_t)(ntile0 + tn) * KT + t * 2 + ks) * 512 + lane * 8);
  };

  f32x4_t acc[BM / 16][TN];
#pragma unroll
  for (int rb = 0; rb < BM / 16; ++rb)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[rb][tn] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  load_a(0);
  load_b(bcur, 0);
  store_a(0);
  __syncthreads();

  for (int t = 0; t < NKT; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < NKT;
    if (more) {
      load_a(t + 1);
      load_b(bnext, t + 1);
    }
    const unsigned char* base = smem + cur * (BM * BK * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int rb = 0; rb < BM / 16; ++rb) {
        const int row = rb * 16 + (lane & 15);
        const u32x4_t a = *reinterpret_cast<const u32x4_t*>(base + lds_off(row, ks * 4 + (lane >> 4)));
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[rb][tn] = mfma16(a, bcur[ks][tn], acc[rb][tn]);
      }
    }
    if (more) {
      store_a(cur ^ 1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) bcur[ks][tn] = bnext[ks][tn];
    }
    __syncthreads();
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
            if (gm < M) epi_qkv_store(ep, gm, col, v, vp);
          } else if (gm < M) {
            if (EPI == EPI_STORE)
              ep.out[(size_t)gm * ep.ldo + col] = f2bf(v);
            else if (EPI == EPI_RESID)
              ep.out[(size_t)gm * ep.ldo + col] = f2bf(bf2f(ep.resid[(size_t)gm * ep.ldr + col]) + v);
          }
        }
      }
    }
  }
}

template <int TN, int EPI>
int launch(const bf16_raw* A, int lda, const bf16_raw* wp, int M, int N, int K, const EpiArgs& ep,
           hipStream_t s) {
  const int MT = (M + BM - 1) / BM, CT = N / (16 * GWAVES * TN);
  gemm_packed_kernel<TN, EPI><<<MT * CT, GTHR, 0, s>>>(A, lda, wp, M, N, K, ep);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

}  // namespace

extern "C" int lsa_gemm(const void* a, int lda, const void* wp, int M, int N, int K, int epi,
                        const EpiArgs* ep, int tn, hipStream_t stream) {
  if (M < 1 || K % BK || lda < K) return LSA_BAD_SHAPE;
  if (tn != 1 && tn != 2) return LSA_UNSUPPORTED;
  if (N % (16 * GWAVES * tn)) return LSA_BAD_SHAPE;
  const bf16_raw* A = static_cast<const bf16_raw*>(a);
  const bf16_raw* W = static_cast<const bf16_raw*>(wp);
  switch (epi) {
    case EPI_STORE:
      return tn == 2 ? launch<2, EPI_STORE>(A, lda, W, M, N, K, *ep, stream) : launch<1, EPI_STORE>(A, lda, W, M, N, K, *ep, stream);
    case EPI_RESID:
      return tn == 2 ? launch<2, EPI_RESID>(A, lda, W, M, N, K, *ep, stream) : launch<1, EPI_RESID>(A, lda, W, M, N, K, *ep, stream);
    case EPI_QKV:
      return tn == 2 ? launch<2, EPI_QKV>(A, lda, W, M, N, K, *ep, stream) : launch<1, EPI_QKV>(A, lda, W, M, N, K, *ep, stream);
    case EPI_SWIGLU:
      if (tn != 2) return LSA_BAD_SHAPE;
      return launch<2, EPI_SWIGLU>(A, lda, W, M, N, K, *ep, stream);
    default: return LSA_UNSUPPORTED;
  }
}
