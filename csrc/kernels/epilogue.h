// Fused GEMM epilogues shared by the decode GEMV (gemv.hip) and the prefill GEMM (gemm.hip).
//
// They replace separate elementwise launches of the reference's HF layer
// (/root/reference/utils/shard_loader.py:66-74 -> LlamaDecoderLayer):
//   EPI_STORE   y -> bf16 out (optionally act(y + bias): GPT-2 c_fc + gelu_new)
//   EPI_RESID   out = resid + y (+ bias)        (o_proj / down_proj + residual add)
//   EPI_SWIGLU  out = silu(gate) * up           (gate/up fused GEMM, tiles interleaved)
//   EPI_QKV     half-split RoPE on q/k + direct write of k/v into the static KV cache
//               (replaces apply_rotary_pos_emb + DynamicCache.update's torch.cat); with
//               cos_t == nullptr (GPT-2: learned absolute positions) no rotation and the
//               natural (unpermuted) column order
// Every mode adds the fp32 per-column ``bias`` first when it is non-null (GPT-2 Conv1D biases).
//   EPI_ARGMAX  greedy argmax over the vocab via 64-bit atomicMax keys
//               (lm_head + torch.argmax, node_worker.py:262-264, fused)
#pragma once
#include "common.h"

// EPI_PARTIAL (gemm_sk only): every K-split workgroup stores its fp32 partial tile to
// ((float*)out)[split][M][ldo]; the following norm kernel adds the partials to the residual
// stream (lsa_resid_rmsnorm_partials) instead of an in-GEMM fixup.
enum EpiMode { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_QKV = 3, EPI_ARGMAX = 4, EPI_PARTIAL = 5 };

// Mirrored by llm_sharding_amd/ops/hip.py::EpiArgs (ctypes) - keep field order in sync.
struct EpiArgs {
  bf16_raw* out;            // STORE/RESID/SWIGLU: [M][ldo]; QKV: q output [M][ldo]
  const bf16_raw* resid;    // RESID: [M][ldr] (may alias out)
  bf16_raw* k_cache;        // QKV: [slots][n_kv][t_max][head_dim]
  bf16_raw* v_cache;
  const int* slot;          // QKV: cache slot of row m
  const int* pos;           // QKV: position of row m
  const float* cos_t;       // QKV: [max_pos][head_dim/2]
  const float* sin_t;
  unsigned long long* keys; // ARGMAX: [M] (zeroed before the launch)
  const float* bias;        // optional [N] fp32, indexed by packed column
  int ldo;
  int ldr;
  int n_heads;
  int n_kv;
  int head_dim;
  int t_max;
  int col_offset;           // ARGMAX: vocabulary index of column 0 (vocab-parallel chunks)
  int act;                  // STORE: 0 identity, 1 gelu (tanh form, GPT-2 "gelu_new")
  // fused RMSNorm across GEMMs (gemm_sk only; layout [M][ss_n] fp32, one partial sum of squares
  // per 64 columns of the residual stream): RESID writes the partials of its rounded outputs to
  // ss_out; QKV / SWIGLU scale row m by rsqrt(sum(ss_in[m][:]) / (64 ss_n) + ss_eps) first
  float* ss_out;
  const float* ss_in;
  int ss_n;
  float ss_eps;
};

LSA_DEVICE float silu(float g) { return g / (1.0f + __expf(-g)); }

// 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))), tanh(u) = 1 - 2 / (exp(2u) + 1)
LSA_DEVICE float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (2.0f - 2.0f / (__expf(2.0f * u) + 1.0f));
}

LSA_DEVICE float epi_bias(const EpiArgs& ep, int col) { return ep.bias ? ep.bias[col] : 0.f; }
LSA_DEVICE float epi_act(const EpiArgs& ep, float v) { return ep.act == 1 ? gelu_tanh(v) : v; }

// Store one finished element (row m, packed column n) of an EPI_QKV GEMM. `vp` is the value
// of the RoPE partner column n ^ 8 (same row). The packed q/k row order within a head is
//   tile tt (16 columns): columns 0..7 -> dims 8tt..8tt+7, columns 8..15 -> dims hd/2+8tt..
// so a rotate_half partner pair always lives in one 16-wide tile (see ops/packing.py).
// ``p`` / ``slot_m``: the row's position and cache slot (ep.pos[m], ep.slot[m]), passed in so a
// caller can request them early.
LSA_DEVICE void epi_qkv_store(const EpiArgs& ep, int m, int n, float v, float vp, int p, int slot_m) {
  const int hd = ep.head_dim, sh = __builtin_ctz((unsigned)hd);  // power of two (host-checked)
  const int qs = ep.n_heads << sh, ks = ep.n_kv << sh;
  if (p < 0 || p >= ep.t_max) return;  // never write outside the static cache
  if (ep.cos_t == nullptr) {  // no RoPE: natural column order [q | k | v]
    const int isk = n >= qs, isv = n >= qs + ks;
    const int c0 = n - (isv ? qs + ks : (isk ? qs : 0));
    const int head = c0 >> sh, dim = c0 & (hd - 1);
    if (!isk) {
      ep.out[(size_t)m * ep.ldo + c0] = f2bf(v);
    } else {
      const size_t base = ((size_t)slot_m * ep.n_kv + head) * ep.t_max + p;
      (isv ? ep.v_cache : ep.k_cache)[base * hd + dim] = f2bf(v);
    }
    return;
  }
  if (n < qs + ks) {
    const bool isq = n < qs;
    const int c0 = isq ? n : n - qs;
    const int head = c0 >> sh, c = c0 & (hd - 1);
    const int tt = c >> 4, cc = c & 15;
    const int half = hd >> 1;
    const int fi = 8 * tt + (cc & 7);
    const int dim = cc < 8 ? fi : half + fi;
    const float cs = ep.cos_t[(size_t)p * half + fi];
    const float sn = ep.sin_t[(size_t)p * half + fi];
    const float r = cc < 8 ? v * cs - vp * sn : v * cs + vp * sn;
    if (isq) {
      ep.out[(size_t)m * ep.ldo + head * hd + dim] = f2bf(r);
    } else {
      const size_t base = ((size_t)slot_m * ep.n_kv + head) * ep.t_max + p;
      ep.k_cache[base * hd + dim] = f2bf(r);
    }
  } else {
    const int c0 = n - qs - ks;
    const int head = c0 >> sh, dim = c0 & (hd - 1);
    const size_t base = ((size_t)slot_m * ep.n_kv + head) * ep.t_max + p;
    ep.v_cache[base * hd + dim] = f2bf(v);
  }
}

// ---------------------------------------------------------------------------------------------
// Vectorised epilogue of one finished 16-column tile row: v[j] = C[m][c0 + j], c0 % 16 == 0
// (packed column order). One thread per (tile, row) instead of one per element: 16-B stores,
// 16-B residual / bias / cos / sin loads, the index math (shifts: head_dim is a power of two)
// done once per 16 outputs. EPI_SWIGLU and EPI_ARGMAX are handled by the callers.
// 16-B store; WT: write-through to memory (two 8-B agent-scope relaxed atomic stores = sc1), so a
// consumer on another CU / XCD may read the bytes after an arrival counter with no release
// fence on this side (MI355X_MICROARCH.md 'Valid forms'; scripts/probes/qkv_attn.hip)
template <bool WT>
LSA_DEVICE void st16x(void* p, u32x4_t v) {
  if constexpr (WT) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, (unsigned long long)v[0] | ((unsigned long long)v[1] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)v[2] | ((unsigned long long)v[3] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    st16(p, v);
  }
}

// ``p`` / ``slot_m``: the row's position and cache slot (ep.pos[m], ep.slot[m]), passed in so a
// caller can request them early (gemv_coop.hip).
template <bool WT = false>
LSA_DEVICE void epi_qkv_row16p(const EpiArgs& ep, int m, int c0, const float* v, int p, int slot_m) {
  const int hd = ep.head_dim, sh = __builtin_ctz((unsigned)hd);
  const int qs = ep.n_heads << sh, ks = ep.n_kv << sh;
  if (p < 0 || p >= ep.t_max) return;  // never write outside the static cache
  const int sec = c0 < qs ? 0 : (c0 < qs + ks ? 1 : 2);
  const int cs0 = c0 - (sec == 0 ? 0 : (sec == 1 ? qs : qs + ks));
  const int head = cs0 >> sh, c = cs0 & (hd - 1);
  bf16_raw* dst = sec == 0 ? ep.out + (size_t)m * ep.ldo + ((size_t)head << sh)
                           : (sec == 1 ? ep.k_cache : ep.v_cache) +
                                 ((((size_t)slot_m * ep.n_kv + head) * ep.t_max + p) << sh);
  if (ep.cos_t == nullptr || sec == 2) {  // v (or no RoPE): natural order, 16 contiguous dims
    st16x<WT>(dst + c, pack8(v));
    st16x<WT>(dst + c + 8, pack8(v + 8));
    return;
  }
  // rotate_half pairs live in this tile: columns 0..7 -> dims 8tt+j, 8..15 -> hd/2 + 8tt + j
  const int half = hd >> 1, fi0 = (c >> 4) * 8;
  const float* ct = ep.cos_t + (size_t)p * half + fi0;
  const float* stb = ep.sin_t + (size_t)p * half + fi0;
  float cs[8], sn[8], lo[8], hi[8];
  *reinterpret_cast<f32x4_t*>(cs) = *reinterpret_cast<const f32x4_t*>(ct);
  *reinterpret_cast<f32x4_t*>(cs + 4) = *reinterpret_cast<const f32x4_t*>(ct + 4);
  *reinterpret_cast<f32x4_t*>(sn) = *reinterpret_cast<const f32x4_t*>(stb);
  *reinterpret_cast<f32x4_t*>(sn + 4) = *reinterpret_cast<const f32x4_t*>(stb + 4);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = v[j] * cs[j] - v[j + 8] * sn[j];
    hi[j] = v[j + 8] * cs[j] + v[j] * sn[j];
  }
  st16x<WT>(dst + fi0, pack8(lo));
  st16x<WT>(dst + half + fi0, pack8(hi));
}

template <bool WT = false>
LSA_DEVICE void epi_qkv_row16(const EpiArgs& ep, int m, int c0, const float* v) {
  epi_qkv_row16p<WT>(ep, m, c0, v, ep.pos[m], ep.slot[m]);
}

// out[m][c0 .. c0+16) = resid (16 bf16 already loaded as two 16-B words) + v
LSA_DEVICE void epi_resid_row16(const EpiArgs& ep, int m, int c0, const float* v, u32x4_t r0, u32x4_t r1) {
  float a[8], b[8];
  unpack8(r0, a);
  unpack8(r1, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] += v[j];
    b[j] += v[j + 8];
  }
  bf16_raw* o = ep.out + (size_t)m * ep.ldo + c0;
  st16(o, pack8(a));
  st16(o + 8, pack8(b));
}

// Adds the bias (if any) to v in place.
LSA_DEVICE void epi_bias16(const EpiArgs& ep, int c0, float* v) {
  if (!ep.bias) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4_t b = *reinterpret_cast<const f32x4_t*>(ep.bias + c0 + 4 * q);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 * q + j] += b[j];
  }
}

template <int EPI>
LSA_DEVICE void epi_row16(const EpiArgs& ep, int m, int c0, float* v) {
  epi_bias16(ep, c0, v);
  if (EPI == EPI_QKV) {
    epi_qkv_row16(ep, m, c0, v);
  } else if (EPI == EPI_STORE) {
    if (ep.act == 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = gelu_tanh(v[j]);
    }
    bf16_raw* o = ep.out + (size_t)m * ep.ldo + c0;
    st16(o, pack8(v));
    st16(o + 8, pack8(v + 8));
  } else if (EPI == EPI_RESID) {
    const bf16_raw* rr = ep.resid + (size_t)m * ep.ldr + c0;
    epi_resid_row16(ep, m, c0, v, ld16(rr), ld16(rr + 8));
  }
}

// Largest argmax key of a 16-column tile row (bias added by epi_bias16 first).
LSA_DEVICE unsigned long long argmax_key16(const float* v, unsigned idx0) {
  unsigned long long k = 0ull;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const unsigned long long kj = argmax_key(v[j], idx0 + j);
    k = kj > k ? kj : k;
  }
  return k;
}
