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
#include "common.h"

namespace {

constexpr int ATT_WAVES = 4;
constexpr int ATT_THR = ATT_WAVES * LSA_WAVE;
constexpr float NEG_BIG = -1e30f;
constexpr int ATT_MAX_SPLIT = 16;  // split-KV factor limit (the merge keeps one lse per split in VGPRs)

// U: key groups in flight per wave per iteration; PF: software-pipelined (the next iteration's
// K/V loads issued before this one's math); NT: non-temporal K/V loads
template <int HD, int G, int U = 4, int PF = 0, int NT = 0>
__global__ __launch_bounds__(ATT_THR) void attn_split_kernel(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc,
    const bf16_raw* __restrict__ vc, const int* __restrict__ slot, const int* __restrict__ pos,
    const int* __restrict__ kv_len, int n_heads, int n_kv, int t_max, float scale_log2,
    int nsplit, int min_chunk, float* __restrict__ part_o, float* __restrict__ part_lse,
    bf16_raw* __restrict__ out, int ldo, unsigned* __restrict__ counters) {
  constexpr int LPK = HD / 8;          // lanes per key row (8 bf16 = 16 B per lane)
  constexpr int KPW = LSA_WAVE / LPK;  // keys per wave-instruction
  constexpr int KPI = KPW * ATT_WAVES; // keys per workgroup iteration

  __shared__ float s_m[ATT_WAVES][G];
  __shared__ float s_l[ATT_WAVES][G];
  __shared__ float s_o[ATT_WAVES][G][HD];
  __shared__ int s_last;

  const int split = blockIdx.x, kvh = blockIdx.y, row = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int grp = lane / LPK, li = lane % LPK;

  int T = kv_len ? kv_len[row] : pos[row] + 1;
  T = T > t_max ? t_max : T;  // never read past the static cache
  int chunk = (T + nsplit - 1) / nsplit;
  chunk = chunk < min_chunk ? min_chunk : chunk;
  chunk = (chunk + KPI - 1) / KPI * KPI;
  const int k0 = split * chunk;
  const int k1 = min(T, k0 + chunk);
  // every split derives the same number of non-empty splits from T: empty ones exit at once
  // (no ticket), and a lone active split writes the final output itself (no merge)
  const int nact = (T + chunk - 1) / chunk;
  if (k0 >= k1) return;
  const size_t pbase = ((size_t)row * n_heads + (size_t)kvh * G) * nsplit + split;
  const __amdgpu_buffer_rsrc_t por = __builtin_amdgcn_make_buffer_rsrc(part_o, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t plr = __builtin_amdgcn_make_buffer_rsrc(part_lse, (short)0, 0x7fffffff, 0x00020000);
  const size_t pbase0 = pbase - split;  // split 0 of head 0 of this group
  // last-arriver merge of the nsplit partials of this (row, kv-head) group (sc1 loads)
  auto combine = [&]() {
    for (int e = tid; e < G * HD; e += ATT_THR) {
      const int r = e / HD, d = e - r * HD;
      const int hb = (int)(pbase0 + (size_t)r * nsplit);  // index of split 0 of head r
      float lse[ATT_MAX_SPLIT];
      float mm = -INFINITY;
#pragma unroll
      for (int sp = 0; sp < ATT_MAX_SPLIT; ++sp) {
        lse[sp] = sp < nact ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(plr, (hb + sp) * 4, 0, 16))
                            : -INFINITY;
        mm = fmaxf(mm, lse[sp]);
      }
      float ws = 0.f, acc = 0.f;
#pragma unroll
      for (int sp = 0; sp < ATT_MAX_SPLIT; ++sp) {
        if (sp < nact) {
          const float wgt = __builtin_amdgcn_exp2f(lse[sp] - mm);
          ws += wgt;
          acc += wgt * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(por, ((hb + sp) * HD + d) * 4, 0, 16));
        }
      }
      out[(size_t)row * ldo + (size_t)(kvh * G + r) * HD + d] = f2bf(acc / ws);
    }
  };
  // publish (every storing wave drained), take the ticket, merge if last
  auto arrive = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* cnt = counters + (size_t)row * n_kv + kvh;
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)(nact - 1);
    }
    __syncthreads();
    if (!s_last) return;
    combine();
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  float qf[G][8];
#pragma unroll
  for (int r = 0; r < G; ++r) {
    unpack8(ld16(q + (size_t)row * ldq + (size_t)(kvh * G + r) * HD + li * 8), qf[r]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[r][j] *= scale_log2;
  }

  const size_t cbase = ((size_t)slot[row] * n_kv + kvh) * (size_t)t_max * HD;
  const bf16_raw* kb = kc + cbase + li * 8;
  const bf16_raw* vb = vc + cbase + li * 8;

  float mx[G], l[G], o[G][8];
#pragma unroll
  for (int r = 0; r < G; ++r) {
    mx[r] = NEG_BIG;
    l[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[r][j] = 0.f;
  }

  auto load = [&](int base_, u32x4_t (&kr_)[U], u32x4_t (&vr_)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = base_ + grp + u * KPI;
      const int kk = key < k1 ? key : k0;
      if (NT) {
        kr_[u] = ld16_nt(kb + (size_t)kk * HD);
        vr_[u] = ld16_nt(vb + (size_t)kk * HD);
      } else {
        kr_[u] = ld16(kb + (size_t)kk * HD);
        vr_[u] = ld16(vb + (size_t)kk * HD);
      }
    }
  };
  u32x4_t kr[U], vr[U];
  if (PF && k0 + w * KPW < k1) load(k0 + w * KPW, kr, vr);
  // loop bound is wave-uniform (the 16-lane key groups of a wave shuffle only internally)
  for (int base = k0 + w * KPW; base < k1; base += KPI * U) {
    u32x4_t kn[U], vn[U];
    if (PF) {
      if (base + KPI * U < k1) load(base + KPI * U, kn, vn);
    } else {
      load(base, kr, vr);
    }
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) valid[u] = base + grp + u * KPI < k1;
    float s[G][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float kf[8];
      unpack8(kr[u], kf);
#pragma unroll
      for (int r = 0; r < G; ++r) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d += qf[r][j] * kf[j];
#pragma unroll
        for (int off = LPK / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
        s[r][u] = valid[u] ? d : NEG_BIG;
      }
    }
#pragma unroll
    for (int r = 0; r < G; ++r) {
      float bm = s[r][0];
#pragma unroll
      for (int u = 1; u < U; ++u) bm = fmaxf(bm, s[r][u]);
      const float mn = fmaxf(mx[r], bm);
      const float alpha = __builtin_amdgcn_exp2f(mx[r] - mn);
      mx[r] = mn;
      l[r] *= alpha;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[r][j] *= alpha;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float p = valid[u] ? __builtin_amdgcn_exp2f(s[r][u] - mn) : 0.f;
        l[r] += p;
        float vf[8];
        unpack8(vr[u], vf);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[r][j] += p * vf[j];
      }
    }
    if (PF) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kr[u] = kn[u];
        vr[u] = vn[u];
      }
    }
  }

  // merge the KPW key-groups of this wave (same li, different grp)
#pragma unroll
  for (int off = LPK; off < LSA_WAVE; off <<= 1) {
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const float mo = __shfl_xor(mx[r], off, 64);
      const float lo = __shfl_xor(l[r], off, 64);
      const float mn = fmaxf(mx[r], mo);
      const float a = __builtin_amdgcn_exp2f(mx[r] - mn), b = __builtin_amdgcn_exp2f(mo - mn);
      l[r] = l[r] * a + lo * b;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[r][j] = o[r][j] * a + __shfl_xor(o[r][j], off, 64) * b;
      mx[r] = mn;
    }
  }
  if (grp == 0) {
#pragma unroll
    for (int r = 0; r < G; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_o[w][r][li * 8 + j] = o[r][j];
      if (li == 0) {
        s_m[w][r] = mx[r];
        s_l[w][r] = l[r];
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < G * HD; e += ATT_THR) {
    const int r = e / HD, d = e - r * HD;
    float mm = s_m[0][r];
#pragma unroll
    for (int i = 1; i < ATT_WAVES; ++i) mm = fmaxf(mm, s_m[i][r]);
    float ls = 0.f, os = 0.f;
#pragma unroll
    for (int i = 0; i < ATT_WAVES; ++i) {
      const float a = __builtin_amdgcn_exp2f(s_m[i][r] - mm);
      ls += s_l[i][r] * a;
      os += s_o[i][r][d] * a;
    }
    if (nact == 1) {  // lone active split: final output directly, no merge
      out[(size_t)row * ldo + (size_t)(kvh * G + r) * HD + d] = f2bf(os / ls);
    } else {
      const int pi = (int)(pbase + (size_t)r * nsplit);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(os / ls), por, (pi * HD + d) * 4, 0, 16 /* sc1 */);
      if (d == 0) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mm + log2f(ls)), plr, pi * 4, 0, 16);
    }
  }
  if (nact > 1) arrive();
}

int g_attn_variant = 0;  // probe knob (scripts/attn_probe.py): 0 = default (U=4, NT), else U*100 + PF*10 + NT

template <int HD, int G, int U, int PF, int NT>
int launch_split_v(const bf16_raw* q, int ldq, const bf16_raw* kc, const bf16_raw* vc, const int* slot,
                   const int* pos, const int* kv_len, int rows, int n_heads, int n_kv, int t_max,
                   float scale_log2, int nsplit, int min_chunk, float* po, float* pl, bf16_raw* out,
                   int ldo, unsigned* cnt, hipStream_t s) {
  dim3 grid(nsplit, n_kv, rows);
  attn_split_kernel<HD, G, U, PF, NT><<<grid, ATT_THR, 0, s>>>(q, ldq, kc, vc, slot, pos, kv_len, n_heads, n_kv,
                                                               t_max, scale_log2, nsplit, min_chunk, po, pl, out, ldo, cnt);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

template <int HD, int G>
int launch_split(const bf16_raw* q, int ldq, const bf16_raw* kc, const bf16_raw* vc, const int* slot,
                 const int* pos, const int* kv_len, int rows, int n_heads, int n_kv, int t_max,
                 float scale_log2, int nsplit, int min_chunk, float* po, float* pl, bf16_raw* out,
                 int ldo, unsigned* cnt, hipStream_t s) {
  if (HD == 128 && G == 1 && g_attn_variant) {
#define LSA_V(UU, P, N)                                                                                    \
  if (g_attn_variant == UU * 100 + P * 10 + N)                                                           \
    return launch_split_v<HD, G, UU, P, N>(q, ldq, kc, vc, slot, pos, kv_len, rows, n_heads, n_kv, t_max, \
                                           scale_log2, nsplit, min_chunk, po, pl, out, ldo, cnt, s);
    LSA_V(2, 0, 0) LSA_V(2, 1, 0) LSA_V(4, 0, 0) LSA_V(4, 1, 0) LSA_V(4, 1, 1) LSA_V(8, 0, 0) LSA_V(8, 0, 1)
    LSA_V(8, 1, 0) LSA_V(6, 0, 0) LSA_V(8, 1, 1) LSA_V(2, 1, 1) LSA_V(2, 0, 1)
#undef LSA_V
  }
  // default: U = 4 groups in flight, non-temporal K/V loads (each cache line is read once per
  // step; 512 x 143-token 7B decode: 5.95 -> 6.79 TB/s, profiles/r2_attn_decode_variants.jsonl)
  return launch_split_v<HD, G, 4, 0, 1>(q, ldq, kc, vc, slot, pos, kv_len, rows, n_heads, n_kv, t_max, scale_log2,
                                        nsplit, min_chunk, po, pl, out, ldo, cnt, s);
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

extern "C" int lsa_attn_set_variant(int v) {
  g_attn_variant = v;
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
