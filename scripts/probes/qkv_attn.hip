// Fused head of a small-batch decode layer: the QKV projection (GEMV with the fused RMSNorm,
// RoPE and KV-cache append) and the attention over the static KV cache in ONE launch.
//
// Why: at batch 1 the attention of a 7B layer reads ~2.5 MB of K/V and is pure latency (6.4 us
// per layer in the decode graph, plus a ~1.2 us kernel boundary: profiles/r4_b1_decode_kernels.txt),
// while the qkv GEMV in front of it streams 100 MB. Here the attention of kv group g starts as
// soon as the q / k / v tiles of group g have been stored, inside the same grid:
//  * blocks [0, n_prod): the GEMV of gemv_body.h (one workgroup per TN 16-column tiles). A
//    workgroup's tiles belong to exactly one kv group g ((head_dim / 16) % TN == 0); its q / k /
//    v stores are write-through (sc1, 16 B), so once they are drained it adds 1 to sync[g] (no
//    release fence: MI355X_MICROARCH.md 'Valid forms', sc1 stores + consumer acquire).
//  * blocks [n_prod, n_prod + rows * n_kv): one attention workgroup per (row, kv group). It
//    polls sync[g] (one lane, relaxed agent loads, s_sleep) until all (G + 2) * head_dim / 16 /
//    TN producers of group g arrived, acquires (agent) and runs the split-KV attention body of
//    attn_body.h on the whole key range (nsplit 1: no partials, no merge).
// Deadlock freedom: consumers have the highest block ids and wait only on lower ones, which
// the dispatcher has placed before them; every wait is also bounded (~20 ms of s_memrealtime):
// a timed-out consumer sets the sticky error word `err` (the host raises on it) and proceeds,
// so the grid always drains. The last consumer of group g to pass its wait zeroes sync[g] and
// its own counter sync[n_kv + g]: every launch starts from zeroed counters (graph-replay safe).
// Reference ops: q/k/v Linear + apply_rotary_pos_emb + DynamicCache.update + eager attention of
// HF LlamaDecoderLayer (/root/reference/utils/shard_loader.py:66-74).
#include "attn_body.h"
#include "gemv_body.h"

// Diagnostic build only (-DLSA_QA_STAMPS, scripts/probes/qa_stamps.py): per-workgroup
// s_memrealtime stamps (100 MHz) written by thread 0 to a buffer nothing else reads:
// 0 start, 1 producer GEMV done / consumer wait done, 2 end. The production library never
// defines it.
#ifdef LSA_QA_STAMPS
__device__ unsigned long long* g_qa_stamps;
#define LSA_QSTAMP(slot)                                                                                     \
  do {                                                                                                      \
    if (threadIdx.x == 0 && g_qa_stamps) g_qa_stamps[blockIdx.x * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LSA_QSTAMP(slot) \
  do {                   \
  } while (0)
#endif

namespace {

constexpr long long QA_SPIN_TICKS = 2000000;  // 20 ms at the 100 MHz s_memrealtime clock
// Counter layout: one 4 KiB page per counter. Packed counters (two cache lines for all of them)
// made every consumer's poll and every producer's arrival hit one memory channel: the channel
// camping slowed the GEMV's weight stream on that channel (producers 21 / 31 us median / max
// instead of 16 / 19 with no consumers; scripts/probes/qa_stamps.py).
#ifndef QA_CSTRIDE
#define QA_CSTRIDE 1024
#endif
#ifndef QA_SLEEP
#define QA_SLEEP 8
#endif
// key groups in flight per wave in the consumer's attention loop (attn_body.h U)
#ifndef QA_U
#define QA_U 4
#endif
#ifndef QA_PF
#define QA_PF 0
#endif

LSA_DEVICE int qa_group_of_tile(int t, int n_heads, int n_kv, int G, int tph) {
  const int qt = n_heads * tph, kt = n_kv * tph;
  if (t < qt) return (t / tph) / G;
  if (t < qt + kt) return (t - qt) / tph;
  return (t - qt - kt) / tph;
}

template <int TN, int U, int G, int HD>
__global__ __launch_bounds__(ATT_THR) void qkv_attn_kernel(const bf16_raw* __restrict__ x, int ldx,
                                                           const bf16_raw* __restrict__ wp, int M, int N, int K,
                                                           float eps, EpiArgs ep, int n_prod, float scale_log2,
                                                           bf16_raw* __restrict__ attn_out, int ldo_attn,
                                                           unsigned* __restrict__ sync, int* __restrict__ err) {
  constexpr int TPH = HD / 16;  // 16-column tiles per head
  // global address-space views of the counters: generic pointers become flat_* atomics, and one
  // flat op anywhere in the kernel made hipcc drain vmcnt(0) before every MFMA of the GEMV loop
  // (the standalone GEMV keeps two chunks in flight) - producers ran 1.2-1.8x longer
  using gu32 = __attribute__((address_space(1))) unsigned;
  using gi32 = __attribute__((address_space(1))) int;
  gu32* gsync = (gu32*)sync;
  gi32* gerr = (gi32*)err;
  const int b = blockIdx.x;
  LSA_QSTAMP(0);
  if (b < n_prod) {
    // q / k / v leave by write-through (sc1) 16-B stores: no L2 write-back (release fence) per
    // workgroup - 768 of them at batch 1 made the launch 2x slower than the two it replaces
#ifdef LSA_QA_PLAIN  // diagnostic (qa_stamps.py): plain stores, no arrival
    gemv_packed_body<TN, 1, ATT_WAVES, U, EPI_QKV, true, false>(x, ldx, nullptr, wp, M, N, K, eps, ep, b);
    LSA_QSTAMP(1);
    return;
#endif
    gemv_packed_body<TN, 1, ATT_WAVES, U, EPI_QKV, true, true>(x, ldx, nullptr, wp, M, N, K, eps, ep, b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drained
    __syncthreads();
    if (threadIdx.x == 0) {
      const int g = qa_group_of_tile(b * TN, ep.n_heads, ep.n_kv, G, TPH);
      __hip_atomic_fetch_add(gsync + g * QA_CSTRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    LSA_QSTAMP(1);
    return;
  }
  const int c = b - n_prod;
  const int g = c % ep.n_kv, row = c / ep.n_kv;
  if (threadIdx.x == 0) {
    const unsigned need = (unsigned)((G + 2) * TPH / TN);
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while (__hip_atomic_load(gsync + g * QA_CSTRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
      __builtin_amdgcn_s_sleep(QA_SLEEP);
      if (__builtin_amdgcn_s_memrealtime() - t0 > QA_SPIN_TICKS) {
        ok = 0;
        __hip_atomic_store(gerr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // the last of the M consumers of group g resets both counters for the next launch
    const unsigned old =
        __hip_atomic_fetch_add(gsync + (ep.n_kv + g) * QA_CSTRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ok && old == (unsigned)(M - 1)) {
      __hip_atomic_store(gsync + g * QA_CSTRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gsync + (ep.n_kv + g) * QA_CSTRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the acquire has completed
  __syncthreads();
  LSA_QSTAMP(1);
  attn_split_body<HD, G, QA_U, QA_PF, 1, false>(ep.out, ep.ldo, ep.k_cache, ep.v_cache, ep.slot, ep.pos, nullptr, ep.n_heads,
                                  ep.n_kv, ep.t_max, scale_log2, 1, 1, nullptr, nullptr, attn_out, ldo_attn,
                                  nullptr, 0, g, row);
  LSA_QSTAMP(2);
}

template <int TN, int U, int G>
int qa_launch(const bf16_raw* x, int ldx, const bf16_raw* wp, int M, int N, int K, float eps, const EpiArgs& ep,
              float sl2, bf16_raw* ao, int ldo_attn, unsigned* sync, int* err, hipStream_t s) {
  const int n_prod = N / 16 / TN;
#ifdef LSA_QA_NOCONS  // diagnostic (qa_stamps.py): producers only
  const int grid = n_prod;
#else
  const int grid = n_prod + M * ep.n_kv;
#endif
  qkv_attn_kernel<TN, U, G, 128><<<grid, ATT_THR, 0, s>>>(x, ldx, wp, M, N, K, eps, ep, n_prod, sl2, ao, ldo_attn,
                                                         sync, err);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

template <int TN, int U>
int qa_dispatch_g(int g, const bf16_raw* x, int ldx, const bf16_raw* wp, int M, int N, int K, float eps,
                  const EpiArgs& ep, float sl2, bf16_raw* ao, int ldo_attn, unsigned* sync, int* err, hipStream_t s) {
  switch (g) {
    case 1: return qa_launch<TN, U, 1>(x, ldx, wp, M, N, K, eps, ep, sl2, ao, ldo_attn, sync, err, s);
    case 2: return qa_launch<TN, U, 2>(x, ldx, wp, M, N, K, eps, ep, sl2, ao, ldo_attn, sync, err, s);
    case 3: return qa_launch<TN, U, 3>(x, ldx, wp, M, N, K, eps, ep, sl2, ao, ldo_attn, sync, err, s);
    case 4: return qa_launch<TN, U, 4>(x, ldx, wp, M, N, K, eps, ep, sl2, ao, ldo_attn, sync, err, s);
    case 8: return qa_launch<TN, U, 8>(x, ldx, wp, M, N, K, eps, ep, sl2, ao, ldo_attn, sync, err, s);
    default: return LSA_UNSUPPORTED;
  }
}

}  // namespace

// QKV projection (x [M][ldx] raw residual rows, wp = pack_b(fold_norm(W_qkv, g)): RMSNorm
// applied in-kernel, eps) + RoPE + KV append into ep->k_cache / v_cache at (slot, pos), q into
// ep->out, then the attention of every row and kv group over keys [0, pos] into attn_out
// [M][ldo_attn]. M <= 16, head_dim 128, G = n_heads / n_kv in {1, 2, 3, 4, 8}, GEMV config
// (tn, nw = 4, u) with 8 % tn == 0. sync: lsa_qkv_attn_sync_words(n_kv) zeroed uint32 (left
// zeroed); err: sticky int32 set to 1 if a consumer's wait timed out (its outputs are invalid).
extern "C" int lsa_qkv_attn(const void* x, int ldx, const void* wp, int M, int N, int K, float eps, const EpiArgs* ep,
                            int tn, int nw, int u, float scale, void* attn_out, int ldo_attn, unsigned* sync, int* err,
                            hipStream_t stream) {
  if (!ep || !x || !wp || !attn_out || !sync || !err) return LSA_BAD_SHAPE;
  if (M < 1 || M > 16 || nw != ATT_WAVES || ldx < K || K % 32 || (K >> 5) % u) return LSA_BAD_SHAPE;
  if (ep->head_dim != 128 || ep->n_kv < 1 || ep->n_heads % ep->n_kv) return LSA_UNSUPPORTED;
  if (N != (ep->n_heads + 2 * ep->n_kv) * ep->head_dim || !ep->out || !ep->k_cache || !ep->v_cache || !ep->slot ||
      !ep->pos || ep->ldo < ep->n_heads * ep->head_dim || ldo_attn < ep->n_heads * ep->head_dim)
    return LSA_BAD_SHAPE;
  if (ep->bias || ep->ss_in || ep->ss_out) return LSA_UNSUPPORTED;
  const int g = ep->n_heads / ep->n_kv;
  const float sl2 = scale * 1.4426950408889634f;
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
  bf16_raw* ao = static_cast<bf16_raw*>(attn_out);
#define LSA_QA(T, UU) \
  if (tn == T && u == UU) return qa_dispatch_g<T, UU>(g, xx, ldx, w, M, N, K, eps, *ep, sl2, ao, ldo_attn, sync, err, stream);
  LSA_QA(1, 4) LSA_QA(1, 8) LSA_QA(2, 4)
#undef LSA_QA
  return LSA_UNSUPPORTED;
}

extern "C" int lsa_qkv_attn_sync_words(int n_kv) { return 2 * n_kv * QA_CSTRIDE; }

#ifdef LSA_QA_STAMPS
extern "C" int lsa_qa_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_qa_stamps), &buf, sizeof(buf)) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}
#endif
