// Flash-style prefill attention over the static KV cache (MFMA, gfx950).
//
// Replaces the reference's HF eager attention in prefill (softmax(QK^T/sqrt(d))V with an
// fp32 softmax, GQA by repeat_kv; SURVEY.md §2.3 K7, reference shard_loader.py:57-74 via
// HF LlamaDecoderLayer) with one kernel that never materialises the score matrix.
//
// Work unit: one query tile (<= 64 consecutive positions of ONE sequence, described by the
// host-built tile table) x one query head; 4 waves, 16 query rows per wave. For every 64-key
// block the K block is staged row-major (XOR-swizzled 16-B chunks) and the V block
// transposed (swizzled 8-B key granules) in LDS, then, per wave:
//   S^T[key][row] = K . Q^T     A = K from LDS, B = Q^T held in registers for the whole tile
//   online softmax              the C layout gives each lane ONE query row (lane & 15), so the
//                               running max / sum / rescale are per-lane scalars plus two
//                               cross-lane max/sum steps (xor 16, xor 32)
//   O^T[dim][row] += V^T . P^T  B = P^T straight from the S^T accumulators (bf16), using the
//                               key order k(8g+j) = 16*(j>>2) + 4g + (j&3) inside each 32-key
//                               fragment, which is exactly what lane group g holds; A = V^T
//                               from LDS in the same key order (two 8-B reads per fragment).
// Causal (row at position p sees keys <= p) or, for the reference's unmasked prefill
// (SURVEY.md Q1), every key < kv_len.
#include "common.h"

namespace {

constexpr int BK = 64, NTHR = 256;  // 64-row query tiles: 4 waves x 16 rows

struct PrefillTile {
  int row0, nrows, slot, pos0, kvlen, pad0, pad1, pad2;
};

template <int HD>
LSA_DEVICE int k_off(int key, int c16) {  // K block [BK][HD] bf16, 16-B chunks swizzled per key
  constexpr int NC = HD / 8;  // 16 (256-B rows): key & 15; 8 (128-B rows): (key >> 1) & 7
  const int sw = NC >= 16 ? (key & 15) : ((key >> 1) & (NC - 1));
  return key * (HD * 2) + ((c16 ^ sw) << 4);
}
template <int HD>
LSA_DEVICE int vt_off(int dim, int g8) {  // V^T block [HD][BK] bf16, 8-B (4-key) granules swizzled per dim
  return dim * (BK * 2) + ((g8 ^ (dim & 15)) << 3);
}

template <int HD>
__global__ __launch_bounds__(NTHR) void flash_prefill_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc, const bf16_raw* __restrict__ vc,
    const PrefillTile* __restrict__ tiles, int n_heads, int n_kv, int t_max, float scale_log2, int causal,
    bf16_raw* __restrict__ out, int ldo) {
  constexpr int KF = HD / 32;     // 32-dim fragments of a query/key row
  constexpr int DT = HD / 16;     // 16-dim output tiles
  constexpr int NC = HD / 8;      // 16-B chunks per key row
  constexpr int LPT = BK * NC / NTHR;  // 16-B loads per thread per operand per block
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BK * HD * 2];
  unsigned char* ks = smem;
  unsigned char* vts = smem + BK * HD * 2;

  const PrefillTile tile = tiles[blockIdx.x];
  const int head = blockIdx.y;
  const int kvh = head / (n_heads / n_kv);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, l16 = lane & 15;

  // ---- Q^T fragments for this wave's 16 rows (row = l16), kept for the whole tile
  const int my_row = w * 16 + l16;
  const bool row_ok = my_row < tile.nrows;
  const int my_pos = tile.pos0 + my_row;
  u32x4_t qf[KF];
  {
    const bf16_raw* qrow = q + (size_t)(tile.row0 + (row_ok ? my_row : 0)) * ldq + head * HD;
#pragma unroll
    for (int kf = 0; kf < KF; ++kf) qf[kf] = ld16(qrow + kf * 32 + g * 8);
  }
  const int lim = causal ? min(tile.pos0 + tile.nrows, tile.kvlen) : tile.kvlen;  // keys any row needs
  const int my_lim = causal ? min(my_pos + 1, tile.kvlen) : tile.kvlen;         // keys this row sees
  const int nkb = (lim + BK - 1) / BK;

  const size_t cache_base = ((size_t)tile.slot * n_kv + kvh) * (size_t)t_max * HD;
  const bf16_raw* kb_ptr = kc + cache_base;
  const bf16_raw* vb_ptr = vc + cache_base;

  // staging map: thread -> (key = i*(NTHR/NC) + tid/NC, chunk = tid%NC)
  const int s_key = tid / NC, s_c = tid % NC;
  u32x4_t kr[LPT], vr[LPT];
  auto load_block = [&](int kb) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      int key = kb * BK + i * (NTHR / NC) + s_key;
      key = key < lim ? key : lim - 1;  // clamp: masked anyway, stays inside the cache
      kr[i] = ld16(kb_ptr + (size_t)key * HD + s_c * 8);
      vr[i] = ld16(vb_ptr + (size_t)key * HD + s_c * 8);
    }
  };
  auto store_block = [&]() {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int key = i * (NTHR / NC) + s_key;
      *reinterpret_cast<u32x4_t*>(ks + k_off<HD>(key, s_c)) = kr[i];
      // transpose V: 8 dims of one key -> 8 rows of V^T
      const unsigned* vw = reinterpret_cast<const unsigned*>(&vr[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int dim = s_c * 8 + j;
        const bf16_raw v = (bf16_raw)((j & 1) ? (vw[j >> 1] >> 16) : (vw[j >> 1] & 0xffffu));
        *reinterpret_cast<bf16_raw*>(vts + vt_off<HD>(dim, key >> 2) + (key & 3) * 2) = v;
      }
    }
  };

  f32x4_t o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) o[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  if (nkb > 0) load_block(0);
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();  // previous block's LDS reads are done
    store_block();
    __syncthreads();
    if (kb + 1 < nkb) load_block(kb + 1);

    // S^T = K . Q^T : 4 key tiles of 16
    f32x4_t s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kf = 0; kf < KF; ++kf) {
        const u32x4_t a = *reinterpret_cast<const u32x4_t*>(ks + k_off<HD>(kt * 16 + l16, kf * 4 + g));
        s[kt] = mfma16(a, qf[kf], s[kt]);
      }
    }
    // scale, mask, block row max (this lane: row my_row, keys kb*64 + kt*16 + 4g + r)
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb * BK + kt * 16 + g * 4 + r;
        const float v = key < my_lim ? s[kt][r] * scale_log2 : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    // fully-masked rows so far (m_new = -inf) keep alpha = 1 and p = 0
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[kt][r] - m_use);
        s[kt][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;  // per-lane partial (this lane's keys); reduced at the end
    m_run = m_new;
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] *= alpha;

    // O^T += V^T . P^T over two 32-key fragments
#pragma unroll
    for (int kf2 = 0; kf2 < 2; ++kf2) {
      float pf[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = s[2 * kf2][r];
        pf[4 + r] = s[2 * kf2 + 1][r];
      }
      const u32x4_t b = pack8(pf);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        const int dim = d * 16 + l16;
        const unsigned long long lo =
            *reinterpret_cast<const unsigned long long*>(vts + vt_off<HD>(dim, kf2 * 8 + g));
        const unsigned long long hi =
            *reinterpret_cast<const unsigned long long*>(vts + vt_off<HD>(dim, kf2 * 8 + 4 + g));
        u32x4_t a;
        a[0] = (unsigned)lo;
        a[1] = (unsigned)(lo >> 32);
        a[2] = (unsigned)hi;
        a[3] = (unsigned)(hi >> 32);
        o[d] = mfma16(a, b, o[d]);
      }
    }
  }

  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  if (!row_ok) return;
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16_raw* orow = out + (size_t)(tile.row0 + my_row) * ldo + head * HD;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    // this lane holds O[row][d*16 + 4g + r], r = 0..3
    const unsigned lo = (unsigned)f2bf(o[d][0] * inv) | ((unsigned)f2bf(o[d][1] * inv) << 16);
    const unsigned hi = (unsigned)f2bf(o[d][2] * inv) | ((unsigned)f2bf(o[d][3] * inv) << 16);
    *reinterpret_cast<unsigned long long*>(orow + d * 16 + g * 4) = (unsigned long long)lo | ((unsigned long long)hi << 32);
  }
}

}  // namespace

// tiles: device array of n_tiles PrefillTile {row0, nrows<=64, slot, pos0, kvlen, pad x3}.
extern "C" int lsa_attn_prefill(const void* q, int ldq, const void* kc, const void* vc, const void* tiles, int n_tiles,
                                int n_heads, int n_kv, int head_dim, int t_max, float scale, int causal, void* out,
                                int ldo, hipStream_t stream) {
  if (n_tiles < 1 || n_heads % n_kv || n_heads < 1) return LSA_BAD_SHAPE;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(n_tiles, n_heads), block(NTHR);
  const auto* t = static_cast<const PrefillTile*>(tiles);
  const auto* qq = static_cast<const bf16_raw*>(q);
  const auto* k = static_cast<const bf16_raw*>(kc);
  const auto* v = static_cast<const bf16_raw*>(vc);
  auto* o = static_cast<bf16_raw*>(out);
  if (head_dim == 128)
    flash_prefill_kernel<128><<<grid, block, 0, stream>>>(qq, ldq, k, v, t, n_heads, n_kv, t_max, sl2, causal, o, ldo);
  else if (head_dim == 64)
    flash_prefill_kernel<64><<<grid, block, 0, stream>>>(qq, ldq, k, v, t, n_heads, n_kv, t_max, sl2, causal, o, ldo);
  else
    return LSA_UNSUPPORTED;
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}
