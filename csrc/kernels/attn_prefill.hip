// Flash-style prefill attention over the static KV cache (MFMA, gfx950).
//
// Replaces the reference's HF eager attention in prefill (softmax(QK^T/sqrt(d))V with an
// fp32 softmax, GQA by repeat_kv; SURVEY.md §2.3 K7, reference shard_loader.py:57-74 via
// HF LlamaDecoderLayer) with one kernel that never materialises the score matrix.
//
// Work unit: one query tile of ONE sequence (host-built tile table) x one KV head's group of
// HPW query heads (HPW = G = n_heads / n_kv when it divides 8, else 1): 8 waves, each owning
// 16 query rows of one head (positions (w / HPW) * 16 ..), so a tile holds 128 / HPW
// positions and every staged K/V block serves the whole GQA group (no re-staging per head).
// Per 64-key block:
//   * K and V arrive by LDS-DMA (global_load_lds, 16 B/lane) into an NBUF-deep ring, blocks
//     kb+1 .. kb+NBUF-1 in flight (counted vmcnt) while block kb is computed; one barrier per block. The swizzle is
//     applied on the SOURCE address, so each 1 KiB piece lands lane-linear.
//   * S^T[key][row] = K . Q^T   A = K rows (ds_read_b128, XOR-swizzled rows: conflict-free),
//                               B = Q^T held in registers for the whole tile
//   * online softmax            each lane holds ONE query row's scores (lane & 15): running
//                               max / sum are per-lane scalars + two cross-lane steps
//   * O^T[dim][row] += V^T . P^T  B = P^T straight from the S^T accumulators (bf16) with the
//                               key order k(8g+j) = 16*(j>>2) + 4g + (j&3) of each 32-key
//                               fragment; A = V^T read with ds_read_b64_tr_b16 (hardware
//                               transpose) from the row-major V image - no transposing stores.
// Causal (row at position p sees keys <= p) or, for the reference's unmasked prefill
// (SURVEY.md Q1), every key < kv_len. Waves skip blocks wholly above their rows' diagonal.
#include "common.h"

namespace {

constexpr int BKV = 64, NWV = 8, NTHR = NWV * 64;  // 64-key blocks, 8 waves x 16 query rows
// K/V ring depth. 2 (block kb+1 in flight while kb is computed) keeps the workgroup at 64 KiB of
// LDS, two per CU; a 4-deep ring (128 KiB, one per CU) measured 6-16 % slower at S >= 2048
// and no faster at S = 512 (scripts/prefill_attn_bench.py)
constexpr int NBUF = 2;

struct PrefillTile {
  int row0, nrows, slot, pos0, kvlen, pad0, pad1, pad2;
};

typedef short v4s_t __attribute__((ext_vector_type(4)));

// chunk swizzle of row r (HD = 128: 16 chunks of 16 B per row). ((r & 3) << 2) ^ (((r >> 2) & 3) << 1)
// makes both read patterns conflict-free: the 16-lane ds_read_b128 groups of the K reads (rows
// l16, chunks kf*4 + lane/16) and the 32-lane ds_read_b64_tr_b16 groups of the V^T reads (8 keys x
// the two chunks of a 16-dim tile) each hit 16 distinct 16-B bank slots. (The previous
// ((r & 3) << 2) | ((r >> 2) & 3) only flipped bit 0 for rows 4-7, which the tr reads' chunk
// pairs {2d, 2d+1} absorb: 2.55 conflict cycles per LDS op in profiles/r2_pmc_hot_kernels.txt.)
template <int HD>
LSA_DEVICE int swz(int r) {
  if constexpr (HD == 128) return ((r & 3) << 2) ^ (((r >> 2) & 3) << 1);
  else return (r >> 1) & 7;
}

// byte offset of 16-B chunk ch of row r in a [BKV][HD] bf16 image
template <int HD>
LSA_DEVICE int sw_off(int r, int ch) {
  return r * (HD * 2) + ((ch ^ swz<HD>(r)) << 4);
}

LSA_DEVICE void glds16(const void* src, unsigned char* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
// non-temporal (aux nt): for bytes one workgroup reads once per step (decode K/V). Not for the
// prefill, whose K/V blocks every query tile of the sequence re-reads from L2.
LSA_DEVICE void glds16_nt(const void* src, unsigned char* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 2);
}

template <int HD, int HPW>
__global__ __launch_bounds__(NTHR) void flash_prefill_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc, const bf16_raw* __restrict__ vc,
    const PrefillTile* __restrict__ tiles, int n_heads, int n_kv, int t_max, float scale_log2, int causal,
    bf16_raw* __restrict__ out, int ldo) {
  constexpr int KF = HD / 32;                 // 32-dim fragments of a query/key row
  constexpr int DT = HD / 16;                 // 16-dim output tiles
  constexpr int NC = HD / 8;                  // 16-B chunks per row
  constexpr int BLK = BKV * HD * 2;           // bytes of one K (or V) block
  constexpr int PPW = BLK / 1024 / NWV;       // 1 KiB DMA pieces per wave per operand
  constexpr int RPP = 1024 / (HD * 2);        // rows per piece
  static_assert(PPW >= 1 && NWV % HPW == 0, "geometry");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * 2 * BLK];  // [buffer][K | V]

  // work item -> (tile, head group). XCD-aware when the group count is a multiple of 8: XCD x
  // (= blockIdx.x % 8 in dispatch order) owns groups x, x+8, ... so their K/V blocks stay in
  // its L2, and walks its items tile-major (heaviest tiles of all its groups first)
  const int n_groups = n_heads / HPW, n_tiles = gridDim.x / n_groups;
  int tix, grp;
  if (n_groups % 8 == 0) {
    const int x = blockIdx.x % 8, j = blockIdx.x / 8, ngx = n_groups / 8;
    tix = j / ngx;
    grp = (j % ngx) * 8 + x;
  } else {
    tix = blockIdx.x % n_tiles;
    grp = blockIdx.x / n_tiles;
  }
  const PrefillTile tile = tiles[tix];
  const int G = n_heads / n_kv;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, l16 = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int head = grp * HPW + w % HPW;
  const int kvh = grp * HPW / G;
  const int prow0 = (w / HPW) * 16;

  // ---- Q^T fragments for this wave's 16 rows (row = l16), kept for the whole tile
  const int my_row = prow0 + l16;
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
  const int wave_lim = causal ? min(tile.pos0 + min(prow0 + 16, tile.nrows), tile.kvlen) : tile.kvlen;
  // blocks entirely below every row's limit need no mask (the wave's first row sees the fewest keys)
  const int wave_min_lim = causal ? min(tile.pos0 + prow0 + 1, tile.kvlen) : tile.kvlen;
  const int nkb = (lim + BKV - 1) / BKV;

  const size_t cache_base = ((size_t)tile.slot * n_kv + kvh) * (size_t)t_max * HD;
  const bf16_raw* kb_ptr = kc + cache_base;
  const bf16_raw* vb_ptr = vc + cache_base;

  // DMA of block kb into buffer buf: piece pc covers rows pc*RPP ..; lane -> (row, dest chunk
  // slot); the source chunk is the swizzle's preimage, so the image is sw_off-addressed
  auto stage = [&](int kb, int buf) {
    unsigned char* kd = smem + buf * (2 * BLK);
#pragma unroll
    for (int s = 0; s < PPW; ++s) {
      const int pc = w * PPW + s;
      const int r = pc * RPP + lane / NC, slot = lane % NC;
      const int ch = slot ^ swz<HD>(r);
      const int key = min(kb * BKV + r, lim - 1);  // clamped rows are masked in the softmax
      glds16(kb_ptr + (size_t)key * HD + ch * 8, kd + pc * 1024);
      glds16(vb_ptr + (size_t)key * HD + ch * 8, kd + BLK + pc * 1024);
    }
  };

  f32x4_t o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) o[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  // per-lane LDS offsets, hoisted out of the block loop (the swizzle term of a lane's reads is
  // the same in every block; rows differ by compile-time multiples folded into the reads)
  int k_off[KF], v_off[DT];
#pragma unroll
  for (int kf = 0; kf < KF; ++kf) k_off[kf] = sw_off<HD>(l16, kf * 4 + g);  // + kt * 16 rows
  const int key_lo = 4 * g + (l16 >> 2);                                    // + f2 * 32 (+ 16) rows
#pragma unroll
  for (int d = 0; d < DT; ++d) v_off[d] = sw_off<HD>(key_lo, 2 * d + ((l16 & 3) >> 1)) + 8 * (l16 & 1);

  // prologue: blocks 0 .. NBUF-2 in flight
  for (int b = 0; b < NBUF - 1 && b < nkb; ++b) stage(b, b);
  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb % NBUF;
    // counted wait: this wave's DMA of block kb landed, its later blocks (up to NBUF-2 of them,
    // 2 * PPW instructions each) may stay in flight
    const int later = min(NBUF - 2, nkb - 1 - kb);
    static_assert(NBUF >= 2 && NBUF <= 4, "ring depth");
    if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * 2 * PPW) : "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // ... every wave's; every wave's reads of block kb-1 done
    if (kb + NBUF - 1 < nkb) stage(kb + NBUF - 1, (kb + NBUF - 1) % NBUF);  // into block kb-1's buffer
    if (kb * BKV >= wave_lim) continue;                 // wave-uniform: all keys above the diagonal
    const unsigned char* ks = smem + cur * (2 * BLK);
    const unsigned char* vs = ks + BLK;

    // S^T = K . Q^T : 4 key tiles of 16 (row kt*16 + l16: the swizzle term depends on l16 only)
    f32x4_t s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kf = 0; kf < KF; ++kf) {
        const u32x4_t a = *reinterpret_cast<const u32x4_t*>(ks + kt * 16 * (HD * 2) + k_off[kf]);
        s[kt] = mfma16(a, qf[kf], s[kt]);
      }
    }
    // scale, mask (diagonal / tail blocks only), block row max (this lane: row my_row, keys
    // kb*64 + kt*16 + 4g + r)
    float mx = -INFINITY;
    if ((kb + 1) * BKV <= wave_min_lim) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[kt][r] *= scale_log2;
          mx = fmaxf(mx, s[kt][r]);
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * BKV + kt * 16 + g * 4 + r;
          const float v = key < my_lim ? s[kt][r] * scale_log2 : -INFINITY;
          s[kt][r] = v;
          mx = fmaxf(mx, v);
        }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    // fully-masked rows so far (m_new = -inf) keep alpha = 1 and p = 0
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    // raw v_exp_f32 (arguments <= 0: no range reduction needed; -inf -> 0)
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(s[kt][r] - m_use);
        s[kt][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;  // per-lane partial (this lane's keys); reduced at the end
    // rescale O only when some row's max moved (wave-uniform branch)
    if (__builtin_amdgcn_ballot_w64(m_new != m_run)) {
#pragma unroll
      for (int d = 0; d < DT; ++d) o[d] *= alpha;
    }
    m_run = m_new;

    // O^T += V^T . P^T over two 32-key fragments; V^T by hardware-transposed reads: in each
    // 16-lane group, lane 4q+p addresses key (base + q), dims 4p..4p+3 of the 16-dim tile
#pragma unroll
    for (int f2 = 0; f2 < 2; ++f2) {
      float pf[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = s[2 * f2][r];
        pf[4 + r] = s[2 * f2 + 1][r];
      }
      const u32x4_t b = pack8(pf);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        // rows key_lo + f2*32 (+16): same swizzle term as key_lo (it depends on row & 15 only
        // through row & 3 and (row >> 2) & 3, unchanged by multiples of 16; HD = 64: (row >> 1) & 7)
        const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_t*)(vs + f2 * 32 * (HD * 2) + v_off[d]));
        const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s_t*)(vs + (f2 * 32 + 16) * (HD * 2) + v_off[d]));
        u32x4_t a;
        a[0] = __builtin_bit_cast(u32x2_t, lo)[0];
        a[1] = __builtin_bit_cast(u32x2_t, lo)[1];
        a[2] = __builtin_bit_cast(u32x2_t, hi)[0];
        a[3] = __builtin_bit_cast(u32x2_t, hi)[1];
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

template <int HD, int HPW>
void launch_prefill(const bf16_raw* q, int ldq, const bf16_raw* k, const bf16_raw* v, const PrefillTile* t,
                    int n_tiles, int n_heads, int n_kv, int t_max, float sl2, int causal, bf16_raw* o, int ldo,
                    hipStream_t stream) {
  dim3 grid(n_tiles * (n_heads / HPW)), block(NTHR);
  flash_prefill_kernel<HD, HPW><<<grid, block, 0, stream>>>(q, ldq, k, v, t, n_heads, n_kv, t_max, sl2, causal, o, ldo);
}

template <int HD>
int dispatch_hpw(int hpw, const bf16_raw* q, int ldq, const bf16_raw* k, const bf16_raw* v, const PrefillTile* t,
                 int n_tiles, int n_heads, int n_kv, int t_max, float sl2, int causal, bf16_raw* o, int ldo,
                 hipStream_t stream) {
  switch (hpw) {
    case 1: launch_prefill<HD, 1>(q, ldq, k, v, t, n_tiles, n_heads, n_kv, t_max, sl2, causal, o, ldo, stream); break;
    case 2: launch_prefill<HD, 2>(q, ldq, k, v, t, n_tiles, n_heads, n_kv, t_max, sl2, causal, o, ldo, stream); break;
    case 4: launch_prefill<HD, 4>(q, ldq, k, v, t, n_tiles, n_heads, n_kv, t_max, sl2, causal, o, ldo, stream); break;
    case 8: launch_prefill<HD, 8>(q, ldq, k, v, t, n_tiles, n_heads, n_kv, t_max, sl2, causal, o, ldo, stream); break;
    default: return LSA_UNSUPPORTED;
  }
  return LSA_OK;
}

// ---- GQA decode attention on MFMA ---------------------------------------------------------
// One workgroup per (decode row, KV head): the G = n_heads / n_kv query heads of the group are
// the 16 MFMA columns (G <= 16), so ONE K/V stream serves the whole group and no MFMA row is
// spent on padding query positions. The NW waves split the row's keys into 32-key sub-blocks
// (wave w takes sub-blocks w, w + NW, ...), each wave staging its own K/V sub-blocks by LDS-DMA
// into a private double buffer (no barrier in the loop: the issuing wave's counted vmcnt orders
// its own reads), computing S^T[key][head] = K . Q^T and O^T += V^T . P^T exactly like the
// prefill kernel (same swizzled images, same permuted key order for P^T), and the NW partial
// (max, sum, O) states are merged through LDS at the end. Keys [0, kv_len or pos + 1) of the
// row's cache slot, tile derived on the device (graph-replay safe).
template <int HD, int NW>
__global__ __launch_bounds__(NW * 64) void gqa_decode_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc, const bf16_raw* __restrict__ vc,
    const int* __restrict__ dslot, const int* __restrict__ dpos, const int* __restrict__ dkvlen, int n_heads,
    int n_kv, int t_max, float scale_log2, bf16_raw* __restrict__ out, int ldo) {
  constexpr int SB = 32;                       // keys per sub-block (one 32-deep PV fragment)
  constexpr int KF = HD / 32, DT = HD / 16, NC = HD / 8;
  constexpr int BLK = SB * HD * 2;             // bytes of one K (or V) sub-block
  constexpr int PPW = BLK / 1024;              // 1 KiB DMA pieces per V sub-block
  constexpr int RPP = 1024 / (HD * 2);         // rows per piece
  constexpr int NKL = 2 * KF;                  // K fragment loads per lane and sub-block
  constexpr int WREG = 2 * BLK;                // one wave's staging: [buffer] V only
  constexpr int MERGE = NW * (16 * HD + 32) * 4;
  constexpr int SMEM = NW * WREG > MERGE ? NW * WREG : MERGE;
  static_assert(PPW >= 1, "geometry");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];

  const int row = blockIdx.x / n_kv, kvh = blockIdx.x % n_kv;
  const int G = n_heads / n_kv;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, l16 = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slot = dslot[row];
  int kl = dkvlen ? dkvlen[row] : dpos[row] + 1;
  kl = kl < t_max ? kl : t_max;  // never read past the static cache
  const bool col_ok = l16 < G;   // MFMA column l16 = query head kvh * G + l16

  // Q^T fragments (B operand): lane holds Q[head l16][kf*32 + 8g .. +7]
  u32x4_t qf[KF];
  {
    const bf16_raw* qrow = q + (size_t)row * ldq + (size_t)(kvh * G + (col_ok ? l16 : 0)) * HD;
#pragma unroll
    for (int kf = 0; kf < KF; ++kf) qf[kf] = col_ok ? ld16(qrow + kf * 32 + g * 8) : u32x4_t{0u, 0u, 0u, 0u};
  }
  const size_t cache_base = ((size_t)slot * n_kv + kvh) * (size_t)t_max * HD;
  const bf16_raw* kb_ptr = kc + cache_base;
  const bf16_raw* vb_ptr = vc + cache_base;
  unsigned char* my = smem + w * WREG;

  // Sub-block sb: V by LDS-DMA into this wave's buffer `buf` (the PV MFMA reads it transposed),
  // K straight into registers - the S^T MFMA's A operand is 16 contiguous bytes of one key row
  // per lane (key kt*16 + l16, dims kf*32 + 8g ..) - so the wave stages half the LDS bytes and a
  // CU holds twice the waves (every byte is read once per step: non-temporal).
  auto stage = [&](int sb, int buf, u32x4_t (&kr)[2][KF]) {
    unsigned char* vd = my + buf * BLK;
#pragma unroll
    for (int s = 0; s < PPW; ++s) {
      const int r = s * RPP + lane / NC, cs = lane % NC;
      const int ch = cs ^ swz<HD>(r);
      const int key = min(sb * SB + r, kl - 1);  // clamped rows are masked in the softmax
      glds16_nt(vb_ptr + (size_t)key * HD + ch * 8, vd + s * 1024);
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int key = min(sb * SB + kt * 16 + l16, kl - 1);
#pragma unroll
      for (int kf = 0; kf < KF; ++kf) kr[kt][kf] = ld16_nt(kb_ptr + (size_t)key * HD + kf * 32 + g * 8);
    }
  };

  f32x4_t o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) o[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  int v_off[DT];
  const int key_lo = 4 * g + (l16 >> 2);
#pragma unroll
  for (int d = 0; d < DT; ++d) v_off[d] = sw_off<HD>(key_lo, 2 * d + ((l16 & 3) >> 1)) + 8 * (l16 & 1);

  // one sub-block: K from registers kr, V from buffer buf
  auto compute = [&](int sb, int buf, const u32x4_t (&kr)[2][KF]) {
    const unsigned char* vs = my + buf * BLK;
    f32x4_t s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kf = 0; kf < KF; ++kf) s[kt] = mfma16(kr[kt][kf], qf[kf], s[kt]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = sb * SB + kt * 16 + g * 4 + r;
        const float v = key < kl ? s[kt][r] * scale_log2 : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = __builtin_amdgcn_exp2f(s[kt][r] - m_use);
        s[kt][r] = pv;
        psum += pv;
      }
    l_run = l_run * alpha + psum;
    if (__builtin_amdgcn_ballot_w64(m_new != m_run)) {
#pragma unroll
      for (int d = 0; d < DT; ++d) o[d] *= alpha;
    }
    m_run = m_new;
    float pf[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pf[r] = s[0][r];
      pf[4 + r] = s[1][r];
    }
    const u32x4_t b = pack8(pf);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s_t*)(vs + v_off[d]));
      const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) v4s_t*)(vs + 16 * (HD * 2) + v_off[d]));
      u32x4_t a;
      a[0] = __builtin_bit_cast(u32x2_t, lo)[0];
      a[1] = __builtin_bit_cast(u32x2_t, lo)[1];
      a[2] = __builtin_bit_cast(u32x2_t, hi)[0];
      a[3] = __builtin_bit_cast(u32x2_t, hi)[1];
      o[d] = mfma16(a, b, o[d]);
    }
  };

  // Two register / LDS buffers alternate with compile-time indices (the loop is unrolled by 2);
  // before reading sub-block sb the wave restages the other buffer with sb + NW (its previous
  // contents were consumed by the previous step) and waits until only the later stage's
  // PPW + NKL operations are in flight: the WHOLE older stage (V DMA and K loads) has retired,
  // whatever order the compiler issued its V DMA and K loads in (compute() needs the K
  // registers first anyway, so waiting for them here costs nothing; advisor round 5).
  const int nsb = (kl + SB - 1) / SB;
  u32x4_t k0r[2][KF], k1r[2][KF];
  auto step = [&](int sb, int cur, u32x4_t (&kcur)[2][KF], u32x4_t (&knext)[2][KF]) {
    if (sb + NW < nsb) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the other buffer's V reads retired
      __builtin_amdgcn_sched_barrier(0);
      stage(sb + NW, cur ^ 1, knext);
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PPW + NKL) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    compute(sb, cur, kcur);
  };
  int sb = w;
  if (sb < nsb) stage(sb, 0, k0r);
  for (; sb < nsb; sb += 2 * NW) {
    step(sb, 0, k0r, k1r);
    if (sb + NW >= nsb) break;
    step(sb + NW, 1, k1r, k0r);
  }
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);

  // merge the NW partial states through LDS: per wave O^T[dim][head] (fp32), m[head], l[head]
  __syncthreads();  // every wave is done with its staging buffers
  float* Ow = reinterpret_cast<float*>(smem);           // [NW][16 heads][HD]
  float* mw = Ow + NW * 16 * HD;                          // [NW][16]
  float* lw = mw + NW * 16;                               // [NW][16]
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int r = 0; r < 4; ++r) Ow[(w * 16 + l16) * HD + d * 16 + 4 * g + r] = o[d][r];
  if (g == 0) {
    mw[w * 16 + l16] = m_run;
    lw[w * 16 + l16] = l_run;
  }
  __syncthreads();
  // 8 output dims per thread-unit: units (head < G, dim octet)
  for (int u = tid; u < G * (HD / 8); u += NW * 64) {
    const int hh = u / (HD / 8), d0 = (u % (HD / 8)) * 8;
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < NW; ++i) M = fmaxf(M, mw[i * 16 + hh]);
    const float Mu = M == -INFINITY ? 0.f : M;
    float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const float f = __builtin_amdgcn_exp2f(mw[i * 16 + hh] - Mu);
      L += lw[i * 16 + hh] * f;
      const float* src = Ow + (i * 16 + hh) * HD + d0;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += src[j] * f;
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    st16(out + (size_t)row * ldo + (size_t)(kvh * G + hh) * HD + d0, pack8(acc));
  }
}

template <int HD>
int launch_gqa_decode(int nw, const bf16_raw* q, int ldq, const bf16_raw* k, const bf16_raw* v, const int* slot,
                      const int* pos, const int* kvlen, int rows, int n_heads, int n_kv, int t_max, float sl2,
                      bf16_raw* o, int ldo, hipStream_t stream) {
  dim3 grid(rows * n_kv);
  if (nw == 1)
    gqa_decode_kernel<HD, 1><<<grid, 64, 0, stream>>>(q, ldq, k, v, slot, pos, kvlen, n_heads, n_kv, t_max, sl2, o, ldo);
  else if (nw == 2)
    gqa_decode_kernel<HD, 2><<<grid, 128, 0, stream>>>(q, ldq, k, v, slot, pos, kvlen, n_heads, n_kv, t_max, sl2, o, ldo);
  else if (nw == 4)
    gqa_decode_kernel<HD, 4><<<grid, 256, 0, stream>>>(q, ldq, k, v, slot, pos, kvlen, n_heads, n_kv, t_max, sl2, o, ldo);
  else
    return LSA_UNSUPPORTED;
  return LSA_OK;
}

}  // namespace

// tiles: device array of n_tiles PrefillTile {row0, nrows, slot, pos0, kvlen, pad x3}; nrows <=
// lsa_prefill_tile_rows(n_heads, n_kv) (128 / heads-per-workgroup).
extern "C" int lsa_prefill_tile_rows(int n_heads, int n_kv) {
  if (n_kv < 1 || n_heads % n_kv) return 0;
  const int g = n_heads / n_kv;
  return NTHR / 64 * 16 / ((NWV % g == 0) ? g : 1);
}

extern "C" int lsa_attn_prefill(const void* q, int ldq, const void* kc, const void* vc, const void* tiles, int n_tiles,
                                int n_heads, int n_kv, int head_dim, int t_max, float scale, int causal, void* out,
                                int ldo, hipStream_t stream) {
  if (n_tiles < 1 || n_kv < 1 || n_heads % n_kv || n_heads < 1) return LSA_BAD_SHAPE;
  const float sl2 = scale * 1.4426950408889634f;
  const int g = n_heads / n_kv, hpw = (NWV % g == 0) ? g : 1;
  const auto* t = static_cast<const PrefillTile*>(tiles);
  const auto* qq = static_cast<const bf16_raw*>(q);
  const auto* k = static_cast<const bf16_raw*>(kc);
  const auto* v = static_cast<const bf16_raw*>(vc);
  auto* o = static_cast<bf16_raw*>(out);
  int rc;
  if (head_dim == 128)
    rc = dispatch_hpw<128>(hpw, qq, ldq, k, v, t, n_tiles, n_heads, n_kv, t_max, sl2, causal, o, ldo, stream);
  else if (head_dim == 64)
    rc = dispatch_hpw<64>(hpw, qq, ldq, k, v, t, n_tiles, n_heads, n_kv, t_max, sl2, causal, o, ldo, stream);
  else
    return LSA_UNSUPPORTED;
  if (rc != LSA_OK) return rc;
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

// GQA decode attention on MFMA (gqa_decode_kernel): one workgroup per (decode row, KV head),
// the group's G = n_heads / n_kv query heads (2 <= G <= 16) as the MFMA columns, keys
// [0, kv_len or pos + 1) of the row's cache slot split over ``nw`` (2 / 4) waves, no split over
// workgroups (callers use it when rows x n_kv fills the GPU). Same numerics as the prefill
// kernel (bf16 P for the PV MFMA). ``nw``: 1 / 2 / 4 waves per item (0 = 1: measured fastest at
// 150 keys - 5.0-5.2 TB/s vs 4.4-4.7 with 2 waves and 3.1 with 4, whose 32-key sub-blocks leave
// waves idle - and within 3 % of 4 waves at 1-4k keys: profiles/r3_attn_gqa_decode.jsonl).
extern "C" int lsa_attn_decode_mfma(const void* q, int ldq, const void* kc, const void* vc, const int* slot,
                                    const int* pos, const int* kv_len, int rows, int n_heads, int n_kv, int head_dim,
                                    int t_max, float scale, void* out, int ldo, int nw, hipStream_t stream) {
  if (rows < 1 || n_kv < 1 || n_heads % n_kv || !slot || !pos) return LSA_BAD_SHAPE;
  const int g = n_heads / n_kv;
  if (g < 2 || g > 16) return LSA_UNSUPPORTED;
  if (ldo % 8 || reinterpret_cast<uintptr_t>(out) % 16 || ldq % 8 || reinterpret_cast<uintptr_t>(q) % 16)
    return LSA_BAD_SHAPE;
  const float sl2 = scale * 1.4426950408889634f;
  const auto* qq = static_cast<const bf16_raw*>(q);
  const auto* k = static_cast<const bf16_raw*>(kc);
  const auto* v = static_cast<const bf16_raw*>(vc);
  auto* o = static_cast<bf16_raw*>(out);
  if (nw == 0) nw = 1;
  int rc;
  if (head_dim == 128)
    rc = launch_gqa_decode<128>(nw, qq, ldq, k, v, slot, pos, kv_len, rows, n_heads, n_kv, t_max, sl2, o, ldo, stream);
  else if (head_dim == 64)
    rc = launch_gqa_decode<64>(nw, qq, ldq, k, v, slot, pos, kv_len, rows, n_heads, n_kv, t_max, sl2, o, ldo, stream);
  else
    return LSA_UNSUPPORTED;
  if (rc != LSA_OK) return rc;
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}
