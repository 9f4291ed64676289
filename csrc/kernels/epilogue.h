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

enum EpiMode { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_QKV = 3, EPI_ARGMAX = 4 };

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
LSA_DEVICE void epi_qkv_store(const EpiArgs& ep, int m, int n, float v, float vp) {
  const int hd = ep.head_dim;
  const int qs = ep.n_heads * hd, ks = ep.n_kv * hd;
  const int p = ep.pos[m];
  if (p < 0 || p >= ep.t_max) return;  // never write outside the static cache
  if (ep.cos_t == nullptr) {  // no RoPE: natural column order [q | k | v]
    const int isk = n >= qs, isv = n >= qs + ks;
    const int c0 = n - (isv ? qs + ks : (isk ? qs : 0));
    const int head = c0 / hd, dim = c0 - head * hd;
    if (!isk) {
      ep.out[(size_t)m * ep.ldo + c0] = f2bf(v);
    } else {
      const size_t base = ((size_t)ep.slot[m] * ep.n_kv + head) * ep.t_max + p;
      (isv ? ep.v_cache : ep.k_cache)[base * hd + dim] = f2bf(v);
    }
    return;
  }
  if (n < qs + ks) {
    const bool isq = n < qs;
    const int c0 = isq ? n : n - qs;
    const int head = c0 / hd, c = c0 - head * hd;
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
      const size_t base = ((size_t)ep.slot[m] * ep.n_kv + head) * ep.t_max + p;
      ep.k_cache[base * hd + dim] = f2bf(r);
    }
  } else {
    const int c0 = n - qs - ks;
    const int head = c0 / hd, dim = c0 - head * hd;
    const size_t base = ((size_t)ep.slot[m] * ep.n_kv + head) * ep.t_max + p;
    ep.v_cache[base * hd + dim] = f2bf(v);
  }
}
