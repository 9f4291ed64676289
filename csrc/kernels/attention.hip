// Attention over the static KV cache.
//
// The reference runs HF eager attention (matmul -> fp32 softmax -> matmul, GQA via
// repeat_kv) on a DynamicCache grown by torch.cat every step (SURVEY.md §2.3 K6/K7,
// /root/reference/utils/shard_loader.py:66-74). Here:
//
//  attn_split_kernel  flash-decoding: grid (nsplit, n_kv, rows). One workgroup streams one
//                     contiguous chunk of a (slot, kv-head)'s keys ONCE for the whole GQA
//                     group of query heads (no repeat_kv copies). K/V rows go straight to
//                     VGPRs (16 B/lane, HD/8 lanes per key), scores and the online softmax
//                     run in fp32 in the exp2 domain. Row m attends keys [0, kvlen(m)):
//                     kvlen = pos+1 (causal; decode and prefill alike) unless an explicit
//                     kv_len array is given (the reference's unmasked prefill, Q1).
//                     K/V rows are read with non-temporal loads (streamed once per step).
//                     The split count is fixed per launch (graph-capturable); the chunk is
//                     derived on-device from the current length, so empty splits exit.
//                     With nsplit > 1 every split publishes its (o, lse) partials with
//                     write-through (sc1) stores and takes an agent-scope arrival ticket per
//                     (row, kv-head); the last-arriving split merges all partials in split
//                     order (deterministic) and writes bf16 [rows][n_heads*HD] - no separate
//                     combine launch (cdna_hip_programming.md §5 'In-launch split-K reduction',
//                     sc1 form). The last arriver resets its counter: graph-replay safe.
#include "attn_body.h"

namespace {

template <int HD, int G, int U = 4, int PF = 0, int NT = 0>
__global__ __launch_bounds__(ATT_THR) void attn_split_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc,
    const bf16_raw* __restrict__ vc, const int* __restrict__ slot, const int* __restrict__ pos,
    const int* __restrict__ kv_len, int n_heads, int n_kv, int t_max, float scale_log2,
    int nsplit, int min_chunk, float* __restrict__ part_o, float* __restrict__ part_lse,
    bf16_raw* __restrict__ out, int ldo, unsigned* __restrict__ counters) {
  attn_split_body<HD, G, U, PF, NT>(q, ldq, kc, vc, slot, pos, kv_len, n_heads, n_kv, t_max, scale_log2, nsplit,
                                    min_chunk, part_o, part_lse, out, ldo, counters, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Few (row, kv-head) work items (e.g. batch-1 decode: 32 workgroups on 256 CUs), one split: each
// workgroup's time is its serial chain of dependent HBM round trips (KPI * U keys per trip; 150
// keys took 3 trips with 4 waves x U 4: 6.4 us per layer, profiles/r4_b1_decode_kernels.txt).
// 8 waves x U 8 keep 256 keys of one (row, kv head) in flight: one trip up to 256 keys.
constexpr int ATT_SMALL_NW = 8, ATT_SMALL_U = 8;
int g_att_small_max_wgs = 128;  // rows * n_kv at or below which the small-grid kernel runs (lsa_attn_set_small_max_wgs)

template <int HD, int G>
__global__ __launch_bounds__(ATT_SMALL_NW * LSA_WAVE) void attn_small_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc,
    const bf16_raw* __restrict__ vc, const int* __restrict__ slot, const int* __restrict__ pos,
    const int* __restrict__ kv_len, int n_heads, int n_kv, int t_max, float scale_log2,
    bf16_raw* __restrict__ out, int ldo) {
  attn_split_body<HD, G, ATT_SMALL_U, 0, 1, false, ATT_SMALL_NW>(q, ldq, kc, vc, slot, pos, kv_len, n_heads, n_kv,
                                                               t_max, scale_log2, 1, 1, nullptr, nullptr, out, ldo,
                                                               nullptr, 0, blockIdx.y, blockIdx.z);
}

// U = 4 key groups in flight, non-temporal K/V loads (each cache line is read once per step;
// 512 x 143-token 7B decode: 5.95 -> 6.79 TB/s over the plain-load / other-U variants,
// profiles/r2_attn_decode_variants.jsonl)
template <int HD, int G>
int launch_split(const bf16_raw* q, int ldq, const bf16_raw* kc, const bf16_raw* vc, const int* slot,
                 const int* pos, const int* kv_len, int rows, int n_heads, int n_kv, int t_max,
                 float scale_log2, int nsplit, int min_chunk, float* po, float* pl, bf16_raw* out,
                 int ldo, unsigned* cnt, hipStream_t s) {
  dim3 grid(nsplit, n_kv, rows);
  if constexpr (G <= 4) {  // (G 6 / 8 would spill at U 8: the GQA models' batch-1 keeps the 4-wave kernel)
    if (nsplit == 1 && rows * n_kv <= g_att_small_max_wgs) {
      attn_small_kernel<HD, G><<<grid, ATT_SMALL_NW * LSA_WAVE, 0, s>>>(q, ldq, kc, vc, slot, pos, kv_len, n_heads,
                                                                        n_kv, t_max, scale_log2, out, ldo);
      LSA_CHECK_LAUNCH();
      return LSA_OK;
    }
  }
  attn_split_kernel<HD, G, 4, 0, 1><<<grid, ATT_THR, 0, s>>>(q, ldq, kc, vc, slot, pos, kv_len, n_heads, n_kv, t_max,
                                                             scale_log2, nsplit, min_chunk, po, pl, out, ldo, cnt);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

template <int HD>
int dispatch_g(int g, const bf16_raw* q, int ldq, const bf16_raw* kc, const bf16_raw* vc,
               const int* slot, const int* pos, const int* kv_len, int rows, int n_heads, int n_kv,
               int t_max, float sl2, int nsplit, int min_chunk, float* po, float* pl, bf16_raw* out,
               int ldo, unsigned* cnt, hipStream_t s) {
#define LSA_G(GG) \
  case GG: return launch_split<HD, GG>(q, ldq, kc, vc, slot, pos, kv_len, rows, n_heads, n_kv, t_max, sl2, nsplit, min_chunk, po, pl, out, ldo, cnt, s);
  switch (g) {
    LSA_G(1) LSA_G(2) LSA_G(3) LSA_G(4) LSA_G(6) LSA_G(8)
    default: return LSA_UNSUPPORTED;
  }
#undef LSA_G
}

}  // namespace

// Host-side switch of the small-grid kernel's range (A/B runs; default 128 work items).
extern "C" int lsa_attn_set_small_max_wgs(int n) {
  if (n < 0) return LSA_BAD_SHAPE;
  g_att_small_max_wgs = n;
  return LSA_OK;
}

extern "C" int lsa_attn_decode(const void* q, int ldq, const void* k_cache, const void* v_cache,
                               const int* slot, const int* pos, const int* kv_len, int rows,
                               int n_heads, int n_kv, int head_dim, int t_max, float scale,
                               int nsplit, int min_chunk, float* part_o, float* part_lse,
                               void* out, int ldo, unsigned* counters, hipStream_t stream) {
  // counters: rows * n_kv zero-initialised uint32 (only read when nsplit > 1; left zeroed)
  if (rows < 1 || n_heads % n_kv || nsplit < 1 || nsplit > ATT_MAX_SPLIT || min_chunk < 1) return LSA_BAD_SHAPE;
  if (nsplit > 1 && !counters) return LSA_BAD_SHAPE;
  const int g = n_heads / n_kv;
  const float sl2 = scale * 1.4426950408889634f;
  const bf16_raw* qq = static_cast<const bf16_raw*>(q);
  const bf16_raw* kc = static_cast<const bf16_raw*>(k_cache);
  const bf16_raw* vc = static_cast<const bf16_raw*>(v_cache);
  bf16_raw* o = static_cast<bf16_raw*>(out);
  int rc;
  if (head_dim == 128)
    rc = dispatch_g<128>(g, qq, ldq, kc, vc, slot, pos, kv_len, rows, n_heads, n_kv, t_max, sl2, nsplit, min_chunk, part_o, part_lse, o, ldo, counters, stream);
  else if (head_dim == 64)
    rc = dispatch_g<64>(g, qq, ldq, kc, vc, slot, pos, kv_len, rows, n_heads, n_kv, t_max, sl2, nsplit, min_chunk, part_o, part_lse, o, ldo, counters, stream);
  else
    return LSA_UNSUPPORTED;
  return rc;
}
