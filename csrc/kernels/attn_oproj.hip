// Batch-1 decode: attention + the o projection (with the residual add) in ONE launch, the o
// projection's weight stream overlapped with the attention. Opt-in (StageEngine.ATTN_OPROJ,
// LSA_ATTN_OPROJ=1): measured slower than the two launches, profiles/r6_attn_oproj.md.
//
// At batch 1 the decode attention is a chain of dependent round trips on 32 workgroups (5.7 us a
// layer at 150-200 keys) and the o-projection GEMV streams 32 MiB of weights (7.4 us). Both
// leave most of the chip's bandwidth unused while they run. Run back to back, their times add up.
// Here the o-projection workgroups issue their whole weight slice into registers at launch and
// only the dot products wait for the attention:
//  * workgroups [0, n_kv): the small-grid attention body (attention.hip attn_small_kernel: 8
//    waves, 256 keys per round trip), the output stored write-through (sc1); each then takes one
//    agent-scope arrival ticket;
//  * workgroups [n_kv, grid): 16-column tiles of W_o dealt evenly (one or two per workgroup) over
//    the full K (no K split, so no cross-workgroup reduction): the 8 waves hold the tiles' K/32
//    fragments in registers (non-temporal loads issued first thing), poll the arrival counter
//    (bounded), read the attention output with sc1 loads, reduce, and add the residual
//    (epilogue.h EPI_RESID).
// Why it loses (ablations, LSA_AO_ABLATE): a CU ingests ~17 GB/s of streamed weights whatever its
// wave count, so the o stream can only go as fast as the CUs NOT running attention take it; at
// 7B two tiles (256 KiB) land on 32 of them (14.7 us for the o part alone), and the 256-workgroup
// launch with its shared counters costs ~1.6 us over the attention kernel alone.
// Round 2 tried the other decomposition, (head, column group) workgroups. Its cross-workgroup
// head reduction cost three dependent memory trips, more than the boundary it removed
// (profiles/r2_attn_oproj_fusion_negative.md). Here the only hand-off is the single arrival
// counter.
//
// Deadlock freedom: the grid is at most one workgroup per CU (<= 256 VGPRs: 2 waves per SIMD,
// 8 waves per workgroup), so every workgroup is resident at once, and the attention workgroups
// need nothing from the others. The poll is bounded (sync[2] records a timeout; the outputs are
// then garbage, never a hang). Replay-safe: the last o workgroup to finish resets both counters.
// Reference: /root/reference/utils/shard_loader.py:66-74 (HF attention + o_proj + residual).
#include "attn_body.h"
#include "epilogue.h"

namespace {

// Probe builds only (scripts/probes/build_attn_oproj_ab.sh; csrc/build.py never sets it):
// 1 = weights loaded after the arrival wait, 2 = no wait (overlap without the hand-off; wrong
// results), 3 = no attention work, 4 = no o-projection work.
#ifndef LSA_AO_ABLATE
#define LSA_AO_ABLATE 0
#endif

constexpr int AO_NW = 8;
constexpr int AO_THR = AO_NW * LSA_WAVE;
constexpr int AO_SPIN_LIMIT = 1 << 22;  // ~0.3 s of s_sleep(2) polls

// tiles [0, tc) of this wave's fragments: fragment (t, i) at 1 KiB block f0 + t * KT + i,
// non-temporal (a device function, not a lambda: hipcc can drop a kernel's host stub when a
// buffer builtin sits in a lambda)
template <int TM, int FPW>
__device__ __forceinline__ void ao_load_w(u32x4_t (&wv)[TM][FPW], __amdgpu_buffer_rsrc_t wr, int tc, int f0, int KT,
                                          int lane) {
#pragma unroll
  for (int t = 0; t < TM; ++t)
    if (t < tc)  // workgroup-uniform
#pragma unroll
      for (int i = 0; i < FPW; ++i)
        wv[t][i] = __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 16, (f0 + t * KT + i) * 1024, 2 /* nt */);
}

// FPW: K/32 fragments per wave (K = 256 * FPW); TM: most 16-column tiles per o workgroup
template <int HD, int G, int FPW, int TM>
__global__ __launch_bounds__(AO_THR, 2) void attn_oproj_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc, const bf16_raw* __restrict__ vc,
    const int* __restrict__ slot, const int* __restrict__ pos, const int* __restrict__ kv_len, int n_heads, int n_kv,
    int t_max, float scale_log2, bf16_raw* __restrict__ attn_out, const bf16_raw* __restrict__ wp, int N, EpiArgs ep,
    unsigned* __restrict__ sync) {
  constexpr int K = 256 * FPW, KT = K / 32;
  __shared__ float s_part[AO_NW][TM * 16];
  __shared__ int s_ok;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_attn = n_kv;
  if ((int)blockIdx.x < n_attn) {
    if (LSA_AO_ABLATE != 3)
      attn_split_body<HD, G, 8, 0, 1, false, AO_NW, true>(q, ldq, kc, vc, slot, pos, kv_len, n_heads, n_kv, t_max,
                                                       scale_log2, 1, 1, nullptr, nullptr, attn_out, K, nullptr, 0,
                                                       blockIdx.x, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every write-through store has left this wave
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }

  // ---- o projection: tiles [t0, t0 + tc) dealt evenly (tc <= TM), every fragment of this
  // wave's K slice into registers right away
  const int ob = blockIdx.x - n_attn, n_o = gridDim.x - n_attn, T = N / 16;
  const int t0 = (int)((long)ob * T / n_o), tc = (int)((long)(ob + 1) * T / n_o) - t0;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)attn_out, (short)0, 0x7fffffff, 0x00020000);
  u32x4_t wv[TM][FPW];
  if (LSA_AO_ABLATE != 1 && LSA_AO_ABLATE != 4) ao_load_w(wv, wr, tc, t0 * KT + w * FPW, KT, lane);

  if (tid == 0) {  // bounded poll of the attention's arrivals
    int ok = LSA_AO_ABLATE == 2 || LSA_AO_ABLATE == 4;
    for (int it = 0; it < AO_SPIN_LIMIT && !ok; ++it) {
      if (__hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)n_attn) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) __hip_atomic_fetch_or(&sync[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ok = ok && LSA_AO_ABLATE != 4;
  }
  __syncthreads();
  if (LSA_AO_ABLATE == 1) ao_load_w(wv, wr, tc, t0 * KT + w * FPW, KT, lane);

  // y[n] = sum_k x[k] W[n][k]: lane l holds column l & 15, k = frag * 32 + 8 (l >> 4) + j
  float acc[TM] = {};
  if (s_ok) {
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      const int kt = w * FPW + i;
      const u32x4_t xv = __builtin_amdgcn_raw_buffer_load_b128(xr, (kt * 32 + 8 * (lane >> 4)) * 2, 0, 16 /* sc1 */);
      float xf[8];
      unpack8(xv, xf);
#pragma unroll
      for (int t = 0; t < TM; ++t)
        if (t < tc) {
          float wf[8];
          unpack8(wv[t][i], wf);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[t] = __builtin_fmaf(xf[j], wf[j], acc[t]);
        }
    }
  }
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    acc[t] += lane_xor<16>(acc[t]);
    acc[t] += lane_xor<32>(acc[t]);
    if (lane < 16) s_part[w][t * 16 + lane] = acc[t];
  }
  __syncthreads();
  if (tid == 0) {
    for (int t = 0; t < tc; ++t) {
      float v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        float a = 0.f;
#pragma unroll
        for (int ww = 0; ww < AO_NW; ++ww) a += s_part[ww][t * 16 + c];  // fixed order: deterministic
        v[c] = a;
      }
      if (s_ok) epi_row16<EPI_RESID>(ep, 0, (t0 + t) * 16, v);
    }
    // the last o workgroup to finish resets the counters for the next launch (graph replays)
    const unsigned old = __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)(n_o - 1)) {
      __hip_atomic_store(&sync[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sync[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int ao_n_cu() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    cached[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  return cached[dev];
}

// (head_dim, GQA group, fragments per wave, tiles per o workgroup): Llama-2-7B (K 4096, 256
// tiles + 32 attention workgroups > 256 CUs: two tiles for some), Llama-2-13B (5120), Llama-3.2-3B
// (3072, GQA 3), the tiny test configs (K 256 / 512)
#define LSA_AO_CONFIGS(X) \
  X(128, 1, 16, 2) X(128, 1, 20, 2) X(128, 3, 12, 1) X(64, 2, 1, 1) X(64, 2, 2, 1) X(64, 2, 2, 2) X(64, 1, 2, 1)

}  // namespace

// One decode row (batch 1): attention of q over the cache (small-grid body, one split) into
// attn_out [1][n_heads * head_dim] (write-through), then out = resid + attn_out @ Wo^T through
// ``ep`` (EPI_RESID) with Wo packed-16x32 [N/16][K/32], K = n_heads * head_dim. sync: 4 zeroed
// uint32 (arrivals, consumers, timeout flag; reset by the kernel). The grid is at most one
// workgroup per CU (max_wg, 0 = the CU count; a smaller value for tests), so every workgroup is
// resident at once. LSA_UNSUPPORTED for shapes without an instantiation (the caller then runs
// attention + GEMV).
extern "C" int lsa_attn_oproj(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* slot,
                              const int* pos, const int* kv_len, int n_heads, int n_kv, int head_dim, int t_max,
                              float scale, void* attn_out, const void* wp, int N, int K, const EpiArgs* ep,
                              unsigned* sync, int max_wg, hipStream_t stream) {
  if (n_heads % n_kv || K != n_heads * head_dim || N % 16 || K % 256 || !sync || !ep) return LSA_BAD_SHAPE;
  const int g = n_heads / n_kv, fpw = K / 256, T = N / 16, cap = max_wg > 0 ? std::min(max_wg, ao_n_cu()) : ao_n_cu();
  if (cap - n_kv < 1) return LSA_UNSUPPORTED;
  const int n_o = std::min(T, cap - n_kv), tm = (T + n_o - 1) / n_o;
  if (tm > 2) return LSA_UNSUPPORTED;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(n_kv + n_o), block(AO_THR);
#define LSA_AO(HD_, G_, F_, TM_)                                                                                     \
  if (head_dim == HD_ && g == G_ && fpw == F_ && tm == TM_) {                                                      \
    attn_oproj_kernel<HD_, G_, F_, TM_><<<grid, block, 0, stream>>>(                                                \
        static_cast<const bf16_raw*>(q), ldq, static_cast<const bf16_raw*>(k_cache),                                \
        static_cast<const bf16_raw*>(v_cache), slot, pos, kv_len, n_heads, n_kv, t_max, sl2,                        \
        static_cast<bf16_raw*>(attn_out), static_cast<const bf16_raw*>(wp), N, *ep, sync);                          \
    LSA_CHECK_LAUNCH();                                                                                             \
    return LSA_OK;                                                                                                  \
  }
  LSA_AO_CONFIGS(LSA_AO)
#undef LSA_AO
  return LSA_UNSUPPORTED;
}
