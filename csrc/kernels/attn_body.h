// Body of the split-KV decode attention (attention.hip, design notes there): one workgroup of
// ATT_THR threads streams one contiguous chunk of a (row, kv-head)'s keys for the whole GQA
// group. Shared by attn_split_kernel (attention.hip) and the fused QKV + attention probe
// (scripts/probes/qkv_attn.hip).
#pragma once
#include "common.h"

#include <type_traits>

constexpr int ATT_WAVES = 4;
constexpr int ATT_THR = ATT_WAVES * LSA_WAVE;
constexpr float NEG_BIG = -1e30f;
constexpr int ATT_MAX_SPLIT = 16;  // split-KV factor limit (the merge keeps one lse per split in VGPRs)

// U: key groups in flight per wave per iteration; PF: software-pipelined (the next iteration's
// K/V loads issued before this one's math); NT: non-temporal K/V loads
// SPLIT = false: the caller guarantees nsplit == 1 (one workgroup per (row, kv head), output
// written directly); the partial / merge code is then not compiled in at all.
// NW: waves per workgroup (the caller launches NW * 64 threads). Few (row, kv-head) work items
// (batch-1 decode: 32 workgroups for the whole chip) are latency-bound - one dependent HBM round
// trip per KPI * U keys - so that case takes 8 waves x U 8 = 256 keys per round trip (attention.hip).
// WT: the final output is stored write-through (sc1), for a consumer on another CU / XCD that
// reads it after an arrival counter in the same launch (attn_oproj.hip).
template <int HD, int G, int U = 4, int PF = 0, int NT = 0, bool SPLIT = true, int NW = ATT_WAVES, bool WT = false>
LSA_DEVICE void attn_split_body(
    const bf16_raw* __restrict__ q, int ldq, const bf16_raw* __restrict__ kc,
    const bf16_raw* __restrict__ vc, const int* __restrict__ slot, const int* __restrict__ pos,
    const int* __restrict__ kv_len, int n_heads, int n_kv, int t_max, float scale_log2,
    int nsplit, int min_chunk, float* __restrict__ part_o, float* __restrict__ part_lse,
    bf16_raw* __restrict__ out, int ldo, unsigned* __restrict__ counters, int split, int kvh, int row) {
  constexpr int LPK = HD / 8;          // lanes per key row (8 bf16 = 16 B per lane)
  constexpr int KPW = LSA_WAVE / LPK;  // keys per wave-instruction
  constexpr int KPI = KPW * NW;        // keys per workgroup iteration
  constexpr int NTHR = NW * LSA_WAVE;

  __shared__ float s_m[NW][G];
  __shared__ float s_l[NW][G];
  __shared__ float s_o[NW][G][HD];
  __shared__ int s_last;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int grp = lane / LPK, li = lane % LPK;

  // the row's cache slot and length: two independent scalar loads, issued together (the empty
  // asm keeps the compiler from sinking the slot load behind the length test's branch)
  const int* lenp = kv_len ? kv_len : pos;
  const int slot_r = slot[row], len_r = lenp[row];
  asm volatile("" ::"s"(slot_r), "s"(len_r));
  const size_t cbase = ((size_t)slot_r * n_kv + kvh) * (size_t)t_max * HD;
  const bf16_raw* kb = kc + cbase + li * 8;
  const bf16_raw* vb = vc + cbase + li * 8;
  int T = len_r + (kv_len ? 0 : 1);
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
    for (int e = tid; e < G * HD; e += NTHR) {
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
  // One-split grids (!SPLIT: batch-1 decode, 32 workgroups on the chip) are a chain of dependent
  // round trips: the first trip's K/V loads go out before q is even requested (they need only
  // slot[row] and the length), so q's load overlaps them instead of preceding them.
  if constexpr (!SPLIT) {
    if (k0 + w * KPW < k1) load(k0 + w * KPW, kr, vr);
    __builtin_amdgcn_sched_barrier(0);
  }

  float qf[G][8];
#pragma unroll
  for (int r = 0; r < G; ++r) {
    unpack8(ld16(q + (size_t)row * ldq + (size_t)(kvh * G + r) * HD + li * 8), qf[r]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[r][j] *= scale_log2;
  }

  if (PF && k0 + w * KPW < k1) load(k0 + w * KPW, kr, vr);
  // loop bound is wave-uniform (the 16-lane key groups of a wave shuffle only internally)
  for (int base = k0 + w * KPW; base < k1; base += KPI * U) {
    u32x4_t kn[U], vn[U];
    if (PF) {
      if (base + KPI * U < k1) load(base + KPI * U, kn, vn);
    } else if (SPLIT || base != k0 + w * KPW) {  // (!SPLIT: the first trip was issued above)
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
        d = group_sum<LPK>(d);  // the key's LPK lanes (DPP; common.h)
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

  // merge the KPW key-groups of this wave (same li, different grp): lane ^ LPK ... ^ 32 on DPP /
  // permlane swaps (common.h lane_xor), no LDS crossbar round trips
  auto merge_groups = [&](auto offc) {
    constexpr int OFF = decltype(offc)::value;
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const float mo = lane_xor<OFF>(mx[r]);
      const float lo = lane_xor<OFF>(l[r]);
      const float mn = fmaxf(mx[r], mo);
      const float a = __builtin_amdgcn_exp2f(mx[r] - mn), b = __builtin_amdgcn_exp2f(mo - mn);
      l[r] = l[r] * a + lo * b;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[r][j] = o[r][j] * a + lane_xor<OFF>(o[r][j]) * b;
      mx[r] = mn;
    }
  };
  static_assert(LPK == 8 || LPK == 16, "key lane groups");
  if constexpr (LPK == 8) merge_groups(std::integral_constant<int, 8>{});
  merge_groups(std::integral_constant<int, 16>{});
  merge_groups(std::integral_constant<int, 32>{});
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
  for (int e = tid; e < G * HD; e += NTHR) {
    const int r = e / HD, d = e - r * HD;
    float mm = s_m[0][r];
#pragma unroll
    for (int i = 1; i < NW; ++i) mm = fmaxf(mm, s_m[i][r]);
    float ls = 0.f, os = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const float a = __builtin_amdgcn_exp2f(s_m[i][r] - mm);
      ls += s_l[i][r] * a;
      os += s_o[i][r][d] * a;
    }
    if (!SPLIT || nact == 1) {  // lone active split: final output directly, no merge
      const size_t oi = (size_t)row * ldo + (size_t)(kvh * G + r) * HD + d;
      if constexpr (WT)
        __builtin_amdgcn_raw_buffer_store_b16(f2bf(os / ls),
                                              __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000),
                                              (int)(oi * 2), 0, 16 /* sc1 */);
      else
        out[oi] = f2bf(os / ls);
    } else {
      const int pi = (int)(pbase + (size_t)r * nsplit);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(os / ls), por, (pi * HD + d) * 4, 0, 16 /* sc1 */);
      if (d == 0) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mm + log2f(ls)), plr, pi * 4, 0, 16);
    }
  }
  if constexpr (SPLIT) {
    if (nact > 1) arrive();
  }
}

