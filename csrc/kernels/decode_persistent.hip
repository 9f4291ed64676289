// Persistent batch-1 decode step: ONE launch per generated token runs
// embedding -> every decoder layer -> fused final norm + lm_head + argmax -> token finalise.
//
// Why (batch-1 latency, the reference's only mode: /root/reference/utils/node_worker.py:493-559,
// SURVEY.md §5.8): at batch 1 a layer is 5 weight-streaming kernels; each one pays an HBM
// ramp (first loads ~2 us in flight with nothing arriving) and a tail, so the launched path
// streams at 4.7-5.8 TB/s (profiles/r2_b1_decode_kernels.txt). Here one grid of one
// workgroup per CU walks the phases of the step with a grid barrier between dependent phases,
// and every workgroup issues the weight loads of its NEXT piece of work (next tile, or the
// first tile of the next projection) before its reduction, epilogue and barrier wait, so the
// next phase starts with its first two chunks of weights already in flight.
//
// Phases of a layer (weights packed 16x32 fragments, ops/packing.py; norms folded into W):
//   qkv   GEMV + fused RMSNorm of h + RoPE + KV-cache append      (epilogue.h epi_qkv_store)
//   attn  one workgroup per query head over its kv head's cache; 8 waves split the keys
//   o     GEMV + residual add into h
//   gu    GEMV (gate|up tile pairs) + fused RMSNorm + SwiGLU -> act
//   down  GEMV + residual add into h
// then the head: GEMV + folded final norm + argmax keys, and workgroup 0 finalises the tokens.
//
// GEMV work unit = TPW 16-column tiles (2 for the SwiGLU pairs) x full K; the 8 waves split K
// (8 / TPW ways per tile) and reduce through LDS in a fixed order. The activation row is staged
// in LDS once per phase (its RMS for the fused norms computed there), so the waves' registers
// hold only the two in-flight weight chunks (191 VGPRs, no spills).
//
// Grid barrier: per-workgroup epoch flags (grid_sync below; replay-safe, no reset needed).
// Hand-offs between phases follow cdna_hip_programming.md §6 Guideline 16 in its
// no-fence form: EVERY byte another workgroup reads in this launch (h, q, attn, act, the new
// K/V rows) is stored write-through (sc1) and drained (vmcnt(0)) before the arrival, and EVERY
// load of such bytes is an sc1 load - so no agent-scope release (an L2 write-back) or acquire
// (an L1/L2 invalidate) runs per barrier. Every spin is bounded: a barrier that does not complete
// within ~LSA_SPIN_LIMIT polls sets *err and the kernel exits (no hang if the grid were ever not
// co-resident; the host checks err).
#include "epilogue.h"

namespace {

constexpr int PW = 8;             // waves per workgroup
constexpr int PTHR = PW * 64;
constexpr int PU = 4;             // weight k-fragments (1 KiB each) per pipeline chunk
constexpr int LSA_SPIN_LIMIT = 1 << 22;

// Diagnostic build only (-DLSA_PERSIST_STAMPS, scripts/persist_stamps.py): thread 0 of every
// workgroup writes s_memrealtime (100 MHz) at the phase boundaries of layer 1 into a buffer
// nothing else reads. The production library never defines it.
#ifdef LSA_PERSIST_STAMPS
__device__ unsigned long long* g_pstamps;
#define LSA_PSTAMP(li, slot)                                                                     \
  do {                                                                                           \
    if ((li) == 1 && threadIdx.x == 0 && g_pstamps) g_pstamps[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LSA_PSTAMP(li, slot) \
  do {                      \
  } while (0)
#endif

struct LayerW {                   // device table, one entry per layer of the stage
  const bf16_raw* qkv;
  const bf16_raw* o;
  const bf16_raw* gu;
  const bf16_raw* down;
  bf16_raw* kc;
  bf16_raw* vc;
};

struct PersistArgs {
  const LayerW* layers;
  int n_layers, M, H, I, nh, nkv, hd, t_max;
  float eps, scale_log2;
  const int* slot;
  int* pos;
  const float* cos_t;
  const float* sin_t;
  bf16_raw* h;                    // [M][H] residual stream (stage input when embed == nullptr)
  bf16_raw* q;                    // [M][nh*hd]
  bf16_raw* attn;                 // [M][nh*hd]
  bf16_raw* act;                  // [M][I]
  const bf16_raw* embed;          // token embedding table, or nullptr
  int* tokens;                    // [M] in: this step's ids (embed); out: next ids (head)
  const bf16_raw* head;           // packed lm_head (final norm folded), or nullptr
  int head_n;                     // lm_head rows (multiple of 16)
  unsigned long long* keys;       // [M] argmax keys (zero on entry, reset on exit)
  int* history;                   // [hist_len][hist_stride] or nullptr
  int hist_stride, hist_len;
  int* step_ctr;
  int pos_inc;                    // added to pos at the end of the step
  unsigned* bar;                  // [grid] barrier flags (epochs), zeroed once
  int* err;
};

// lane id recomputed where used (v_mbcnt), so per-lane addresses are not hoisted out of the
// phase loop and kept live across every phase (cdna_hip_programming.md, attention pitfalls)
LSA_DEVICE int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// write-through (sc1) stores / sc1 loads of handed-off data; buffer resources are built from a
// wave-uniform base, the per-lane part stays in the 32-bit offset
LSA_DEVICE __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
LSA_DEVICE void st_b16(bf16_raw* base, int idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)f2bf(v), rsrc(base), idx * 2, 0, 16);
}
LSA_DEVICE void st_b128(void* base, int off, u32x4_t v) { __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), off, 0, 16); }
LSA_DEVICE u32x4_t ld_b128(const void* base, int off) { return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), off, 0, 16); }
LSA_DEVICE float ld_b16f(const bf16_raw* base, int idx) {
  return bf2f((bf16_raw)__builtin_amdgcn_raw_buffer_load_b16(rsrc(base), idx * 2, 0, 16));
}

// ---------------------------------------------------------------------------- grid barrier
// Flag barrier: workgroup g stores the barrier's epoch into flags[g] (one write-through word,
// no atomics: a single contended counter serialises 256 read-modify-writes), and one wave per
// workgroup polls all G flags (4 words per lane, sc1 loads) until every one has reached the
// epoch. Epochs grow by one per barrier across launches (each workgroup starts from its own
// flag, which every workgroup left at the same value), compared mod 2^32.
LSA_DEVICE bool grid_sync(const PersistArgs& a, unsigned& epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's sc1 stores have landed
  __syncthreads();
  __shared__ int s_ok;
  ++epoch;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x, G = gridDim.x;
    if (lane == 0) __hip_atomic_store(a.bar + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1, spins = 0;
    for (;;) {
      bool done = true;
      for (int i = lane; i < G; i += 64)
        done &= (int)(__hip_atomic_load(a.bar + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - epoch) >= 0;
      if (__all(done)) break;
      if (++spins > LSA_SPIN_LIMIT || __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        if (lane == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) s_ok = ok;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps later loads below
  return s_ok != 0;
}

// ---------------------------------------------------------------------------- GEMV phases
enum Phase { PH_QKV = 0, PH_O = 1, PH_GU = 2, PH_DOWN = 3, PH_HEAD = 4 };

struct Job {                      // weight stream of one projection (packed [N/16][K/32][64][8])
  const bf16_raw* w;
  int N, K, tpw;
};

// this wave's share of a unit: tile index and K range [kb, ke) in fragments (whole chunks)
LSA_DEVICE void wave_part(const Job& j, int unit, int w, int& tile, int& kb, int& ke) {
  const int wpt = PW / j.tpw;     // waves per tile
  const int KT = j.K >> 5, nu = KT / PU;
  const int ws = w % wpt;
  tile = unit * j.tpw + w / wpt;
  kb = (ws * nu / wpt) * PU;
  ke = ((ws + 1) * nu / wpt) * PU;
}

LSA_DEVICE void load_w(const bf16_raw* w, int KT, int tile, int kt, int lane, u32x4_t (&b)[PU]) {
  const bf16_raw* p = w + ((size_t)tile * KT + kt) * 512 + lane * 8;
#pragma unroll
  for (int u = 0; u < PU; ++u) b[u] = ld16_nt(p + u * 512);
}

// issue the first two weight chunks of this wave's part of `unit` of `j`
LSA_DEVICE void prefetch(const Job& j, int unit, int w, int lane, u32x4_t (&bA)[PU], u32x4_t (&bB)[PU]) {
  int tile, kb, ke;
  wave_part(j, unit, w, tile, kb, ke);
  const int KT = j.K >> 5;
  if (kb < ke) load_w(j.w, KT, tile, kb, lane, bA);
  if (kb + PU < ke) load_w(j.w, KT, tile, kb + PU, lane, bB);
}

// epi_qkv_store (epilogue.h) for row 0 with write-through stores: q -> a.q, k / v -> the cache
// rows at pos[0] (RoPE rotate_half partner in the same 16-column tile, packed q/k order)
LSA_DEVICE void qkv_store(const PersistArgs& a, const LayerW* L, int n, float v, float vp) {
  const int hd = a.hd, sh = __builtin_ctz((unsigned)hd);
  const int qs = a.nh << sh, ks = a.nkv << sh;
  const int p = a.pos[0];
  if (p < 0 || p >= a.t_max) return;
  if (n < qs + ks) {
    const bool isq = n < qs;
    const int c0 = isq ? n : n - qs;
    const int head = c0 >> sh, c = c0 & (hd - 1);
    const int tt = c >> 4, cc = c & 15, half = hd >> 1;
    const int fi = 8 * tt + (cc & 7);
    const int dim = cc < 8 ? fi : half + fi;
    const float cs = a.cos_t[(size_t)p * half + fi], sn = a.sin_t[(size_t)p * half + fi];
    const float r = cc < 8 ? v * cs - vp * sn : v * cs + vp * sn;
    if (isq) {
      st_b16(a.q, head * hd + dim, r);
    } else {
      bf16_raw* kb = L->kc + (((size_t)a.slot[0] * a.nkv + head) * a.t_max + p) * hd;
      st_b16(kb, dim, r);
    }
  } else {
    const int c0 = n - qs - ks;
    const int head = c0 >> sh, dim = c0 & (hd - 1);
    bf16_raw* vb = L->vc + (((size_t)a.slot[0] * a.nkv + head) * a.t_max + p) * hd;
    st_b16(vb, dim, v);
  }
}

// One unit (TPW tiles x full K) of phase PH; then the prefetch of (nj, nunit) if nj.w.
// M == 1: the activation row sits in LDS (s_x, staged by gemv_phase); MFMA row 0 is the real
// row (lanes l16 == 0 supply it), rows 1..15 are zero.
template <int PH>
LSA_DEVICE void gemv_unit(const PersistArgs& a, const LayerW* L, const Job& j, int unit, u32x4_t (&bA)[PU],
                          u32x4_t (&bB)[PU], const Job& nj, int nunit, float* red, const bf16_raw* s_x, float rs,
                          unsigned long long* s_key) {
  constexpr int TPW = PH == PH_GU ? 2 : 1;
  const int tid = threadIdx.x, lane = lane_id(), kq = lane >> 4, l16 = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int tile, kb, ke;
  wave_part(j, unit, w, tile, kb, ke);
  const int KT = j.K >> 5;
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  const bf16_raw* xs = s_x + 8 * kq;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  auto comp = [&](int kt, const u32x4_t (&b)[PU]) {
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const u32x4_t x8 = l16 == 0 ? *reinterpret_cast<const u32x4_t*>(xs + (kt + u) * 32) : zero;
      acc = mfma16(x8, b[u], acc);
    }
  };
  if (kb < ke) {
    // invariant at the top of each half: the current chunk's weights are in bA (bB), the next
    // chunk's (if any) in bB (bA); weights run two chunks ahead of the MFMAs
    int kt = kb;
    for (;;) {
      comp(kt, bA);
      if (kt + PU >= ke) break;
      if (kt + 2 * PU < ke) load_w(j.w, KT, tile, kt + 2 * PU, lane, bA);
      kt += PU;
      comp(kt, bB);
      if (kt + PU >= ke) break;
      if (kt + 2 * PU < ke) load_w(j.w, KT, tile, kt + 2 * PU, lane, bB);
      kt += PU;
    }
  }
  // the next unit's first weights go out before the reduction / epilogue / barrier
  if (nj.w) prefetch(nj, nunit, w, lane, bA, bB);

  // reduce row 0 only: red[w][col 0..15] (C layout: col = l16, row = 4*kq + r; row 0 = kq 0, r 0)
  if (kq == 0) red[w * 16 + l16] = acc[0];
  __syncthreads();
  constexpr int WPT = PW / TPW;
  if (tid < 16 * TPW) {
    const int t = tid >> 4, n = tid & 15;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < WPT; ++i) v += red[(t * WPT + i) * 16 + n];
    red[PW * 16 + tid] = v * rs;   // reduced, normalised row of the unit's tiles
  }
  __syncthreads();
  const float* rv = red + PW * 16;
  if (tid < 16) {
    const int n = tid, col = unit * 16 + n;
    if (PH == PH_GU) {  // tiles (2u, 2u+1) = (gate, up) of output columns 16u..16u+15
      st_b16(a.act, col, silu(rv[n]) * rv[16 + n]);
    } else if (PH == PH_O || PH == PH_DOWN) {
      st_b16(a.h, col, ld_b16f(a.h, col) + rv[n]);
    } else if (PH == PH_QKV) {
      qkv_store(a, L, col, rv[n], rv[n ^ 8]);
    } else {  // PH_HEAD: largest key of the tile -> one atomic
      unsigned long long k = argmax_key(rv[n], (unsigned)col);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        const unsigned long long ko = __shfl_xor(k, o, 64);
        k = ko > k ? ko : k;
      }
      if (n == 0) __hip_atomic_fetch_max(a.keys, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();  // red reused by the next unit
}

// `have`: bA/bB already hold this workgroup's first chunks of its next unit (prefetched by the
// previous unit); otherwise they are loaded at the start of the unit
template <int PH>
LSA_DEVICE void gemv_phase(const PersistArgs& a, const LayerW* L, const Job& j, const Job& next,
                           u32x4_t (&bA)[PU], u32x4_t (&bB)[PU], float* red, bf16_raw* s_x,
                           unsigned long long* s_key, bool& have) {
  constexpr bool NORM = PH == PH_QKV || PH == PH_GU || PH == PH_HEAD;
  const int units = j.N / 16 / j.tpw;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
  const int G = gridDim.x;
  if ((int)blockIdx.x >= units) return;
  // stage the activation row in LDS (+ its RMS for the fused norm; fixed reduction order)
  const bf16_raw* x = PH == PH_O ? a.attn : (PH == PH_DOWN ? a.act : a.h);
  float ss = 0.f;
  for (int c = threadIdx.x; c < j.K / 8; c += PTHR) {
    const u32x4_t v = ld_b128(x, c * 16);
    *reinterpret_cast<u32x4_t*>(s_x + c * 8) = v;
    if (NORM) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int q = 0; q < 8; ++q) ss += f[q] * f[q];
    }
  }
  float rs = 1.f;
  if (NORM) {
    ss = wave_sum(ss);
    if (lane == 0) red[w] = ss;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < PW; ++i) t += red[i];
    rs = rsqrtf(t / (float)j.K + a.eps);
  }
  __syncthreads();
  for (int u = blockIdx.x; u < units; u += G) {
    if (!have) prefetch(j, u, w, lane, bA, bB);
    Job nj{nullptr, 0, 0, 1};
    int nu = 0;
    if (u + G < units) {
      nj = j;
      nu = u + G;
    } else if (next.w && (int)blockIdx.x < next.N / 16 / next.tpw) {
      nj = next;
      nu = blockIdx.x;
    }
    gemv_unit<PH>(a, L, j, u, bA, bB, nj, nu, red, s_x, rs, s_key);
    have = nj.w != nullptr;
  }
}

// ---------------------------------------------------------------------------- attention
// unit = one query head hq (row 0) against keys [0, pos + 1) of its kv head hq / (nh / nkv)
// (GQA groups re-read their kv head per query head: at batch 1 the cache read is tiny and one
// head per unit keeps the registers of the whole persistent kernel within 256 VGPRs);
// lanes: HD/8 per key (16 B each), 8 waves x (64 / (HD/8)) keys per step, U = 4 steps in flight.
template <int HD>
LSA_DEVICE void attn_unit(const PersistArgs& a, const LayerW& L, int hq, float* sm) {
  constexpr int G = 1, LPK = HD / 8, KPW = 64 / LPK, KPI = KPW * PW, U = 4;
  const int row = 0, kvh = hq / (a.nh / a.nkv);
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6, grp = lane / LPK, li = lane % LPK;
  const int T = min(a.pos[row] + 1, a.t_max);
  const int nh = a.nh;
  float qf[G][8];
#pragma unroll
  for (int r = 0; r < G; ++r) {
    unpack8(ld_b128(a.q, (row * nh * HD + (hq + r) * HD + li * 8) * 2), qf[r]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[r][j] *= a.scale_log2;
  }
  const size_t cb = ((size_t)a.slot[row] * a.nkv + kvh) * (size_t)a.t_max * HD;
  const bf16_raw* kb = L.kc + cb;  // wave-uniform bases; lane part in the sc1 load offsets
  const bf16_raw* vb = L.vc + cb;
  float mx[G], l[G], o[G][8];
#pragma unroll
  for (int r = 0; r < G; ++r) {
    mx[r] = -1e30f;
    l[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[r][j] = 0.f;
  }
  for (int base = w * KPW; base < T; base += KPI * U) {
    u32x4_t kr[U], vr[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = base + grp + u * KPI;
      valid[u] = key < T;
      const int kk = valid[u] ? key : 0;
      kr[u] = ld_b128(kb, (kk * HD + li * 8) * 2);
      vr[u] = ld_b128(vb, (kk * HD + li * 8) * 2);
    }
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
        s[r][u] = valid[u] ? d : -1e30f;
      }
    }
#pragma unroll
    for (int r = 0; r < G; ++r) {
      float bm = s[r][0];
#pragma unroll
      for (int u = 1; u < U; ++u) bm = fmaxf(bm, s[r][u]);
      const float mn = fmaxf(mx[r], bm);
      const float al = __builtin_amdgcn_exp2f(mx[r] - mn);
      mx[r] = mn;
      l[r] *= al;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[r][j] *= al;
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
  }
  // merge the key groups of this wave, then the 8 waves through LDS
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1) {
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const float mo = __shfl_xor(mx[r], off, 64), lo = __shfl_xor(l[r], off, 64);
      const float mn = fmaxf(mx[r], mo);
      const float x1 = __builtin_amdgcn_exp2f(mx[r] - mn), x2 = __builtin_amdgcn_exp2f(mo - mn);
      l[r] = l[r] * x1 + lo * x2;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[r][j] = o[r][j] * x1 + __shfl_xor(o[r][j], off, 64) * x2;
      mx[r] = mn;
    }
  }
  float* s_m = sm;                       // [PW][G]
  float* s_l = sm + PW * G;              // [PW][G]
  float* s_o = sm + 2 * PW * G;          // [PW][G][HD]
  if (grp == 0) {
#pragma unroll
    for (int r = 0; r < G; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_o[(w * G + r) * HD + li * 8 + j] = o[r][j];
      if (li == 0) {
        s_m[w * G + r] = mx[r];
        s_l[w * G + r] = l[r];
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < G * HD; e += PTHR) {
    const int r = e / HD, d = e - r * HD;
    float mm = s_m[r];
#pragma unroll
    for (int i = 1; i < PW; ++i) mm = fmaxf(mm, s_m[i * G + r]);
    float ls = 0.f, os = 0.f;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const float x = __builtin_amdgcn_exp2f(s_m[i * G + r] - mm);
      ls += s_l[i * G + r] * x;
      os += s_o[(i * G + r) * HD + d] * x;
    }
    st_b16(a.attn, row * nh * HD + (hq + r) * HD + d, os / ls);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------- the step
constexpr int MAX_K = 32768;      // longest activation row staged in LDS (hidden / intermediate)

template <int HD>
__global__ __launch_bounds__(PTHR) void decode_persistent_kernel(PersistArgs a) {
  __shared__ float red[PW * 16 + 64];
  __shared__ __attribute__((aligned(16))) bf16_raw s_x[MAX_K];
  __shared__ unsigned long long s_key[16];
  __shared__ float sm[2 * PW + PW * HD];
  const int tid = threadIdx.x;
  const int H = a.H, I = a.I, qs = a.nh * HD, ks = a.nkv * HD;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  u32x4_t bA[PU], bB[PU];
  const Job none{nullptr, 0, 0, 1};

  // embedding of this step's tokens (the residual stream for layer 0)
  if (a.embed) {
    for (int e = blockIdx.x * PTHR + tid; e < a.M * (H / 8); e += gridDim.x * PTHR) {
      const int m = e / (H / 8), c = e - m * (H / 8);
      st_b128(a.h, (m * H + c * 8) * 2, ld16(a.embed + (size_t)a.tokens[m] * H + c * 8));
    }
  }
  unsigned epoch = __hip_atomic_load(a.bar + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool have = false;
  if (a.n_layers > 0) {
    const Job j0{a.layers[0].qkv, qs + 2 * ks, H, 1};
    if ((int)blockIdx.x < j0.N / 16) {
      prefetch(j0, blockIdx.x, w, lane, bA, bB);
      have = true;
    }
  }
  if (a.embed && !grid_sync(a, epoch)) return;

  for (int li = 0; li < a.n_layers; ++li) {
    const LayerW* L = a.layers + li;
    // qkv (no prefetch across the attention phase: it would hold 32 VGPRs through it)
    LSA_PSTAMP(li, 0);
    gemv_phase<PH_QKV>(a, L, Job{L->qkv, qs + 2 * ks, H, 1}, none, bA, bB, red, s_x, s_key, have);
    LSA_PSTAMP(li, 1);
    if (!grid_sync(a, epoch)) return;
    LSA_PSTAMP(li, 2);
    for (int u = blockIdx.x; u < a.nh; u += gridDim.x) attn_unit<HD>(a, *L, u, sm);
    have = false;
    LSA_PSTAMP(li, 3);
    if (!grid_sync(a, epoch)) return;
    LSA_PSTAMP(li, 4);
    gemv_phase<PH_O>(a, L, Job{L->o, H, qs, 1}, Job{L->gu, 2 * I, H, 2}, bA, bB, red, s_x, s_key, have);
    LSA_PSTAMP(li, 5);
    if (!grid_sync(a, epoch)) return;
    LSA_PSTAMP(li, 6);
    gemv_phase<PH_GU>(a, L, Job{L->gu, 2 * I, H, 2}, Job{L->down, H, I, 1}, bA, bB, red, s_x, s_key, have);
    LSA_PSTAMP(li, 7);
    if (!grid_sync(a, epoch)) return;
    LSA_PSTAMP(li, 8);
    const Job nq = li + 1 < a.n_layers ? Job{a.layers[li + 1].qkv, qs + 2 * ks, H, 1}
                                       : (a.head ? Job{a.head, a.head_n, H, 1} : none);
    gemv_phase<PH_DOWN>(a, L, Job{L->down, H, I, 1}, nq, bA, bB, red, s_x, s_key, have);
    LSA_PSTAMP(li, 9);
    if (!grid_sync(a, epoch)) return;
    LSA_PSTAMP(li, 10);
  }
  if (a.head) {
    gemv_phase<PH_HEAD>(a, nullptr, Job{a.head, a.head_n, H, 1}, none, bA, bB, red, s_x, s_key, have);
    if (!grid_sync(a, epoch)) return;
  }
  // finalise (workgroup 0): token ids, key reset, history, positions
  if (blockIdx.x == 0) {
    const int step = a.step_ctr ? *a.step_ctr : 0;
    __syncthreads();
    if (tid < a.M) {
      if (a.head) {
        const unsigned long long k = __hip_atomic_load(a.keys + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int tok = (int)argmax_key_index(k);
        __hip_atomic_store(a.keys + tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.tokens[tid] = tok;
        if (a.history && step < a.hist_len) a.history[(size_t)step * a.hist_stride + tid] = tok;
      }
      a.pos[tid] += a.pos_inc;
    }
    if (tid == 0 && a.step_ctr && a.head) *a.step_ctr = step + 1;
  }
}

template <int HD>
int launch_hd(const PersistArgs& a, int grid, hipStream_t s) {
  decode_persistent_kernel<HD><<<grid, PTHR, 0, s>>>(a);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

}  // namespace

// One decode step of a stage for ONE row (cache slot slot[0] at position pos[0]);
// layers: device array of n_layers {qkv, o, gate_up, down, k_cache, v_cache} pointers (packed
// bf16 weights, norms folded). grid: workgroups (one per CU; every one must be resident at once).
extern "C" int lsa_decode_persistent(const void* layers, int n_layers, int M, int H, int I, int nh, int nkv, int hd,
                                     int t_max, float eps, float scale, const int* slot, int* pos, const float* cos_t,
                                     const float* sin_t, void* h, void* q, void* attn, void* act, const void* embed,
                                     int* tokens, const void* head, int head_n, unsigned long long* keys,
                                     int* history, int hist_stride, int hist_len, int* step_ctr, int pos_inc,
                                     unsigned* bar, int* err, int grid, hipStream_t stream) {
  if (M != 1 || n_layers < 0 || nkv < 1 || nh % nkv || H % 256 || I % 32 || grid < 1 || !bar || !err ||
      H > MAX_K || I > MAX_K)
    return LSA_BAD_SHAPE;
  if ((H / 32) % PU || (I / 32) % PU || (nh * hd / 32) % PU || (head && (head_n % 16 || !keys || !tokens)) ||
      (embed && !tokens))
    return LSA_BAD_SHAPE;
  if (!cos_t || !sin_t) return LSA_UNSUPPORTED;  // Llama family (RoPE) only
  PersistArgs a;
  a.layers = static_cast<const LayerW*>(layers);
  a.n_layers = n_layers;
  a.M = M;
  a.H = H;
  a.I = I;
  a.nh = nh;
  a.nkv = nkv;
  a.hd = hd;
  a.t_max = t_max;
  a.eps = eps;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.slot = slot;
  a.pos = pos;
  a.cos_t = cos_t;
  a.sin_t = sin_t;
  a.h = static_cast<bf16_raw*>(h);
  a.q = static_cast<bf16_raw*>(q);
  a.attn = static_cast<bf16_raw*>(attn);
  a.act = static_cast<bf16_raw*>(act);
  a.embed = static_cast<const bf16_raw*>(embed);
  a.tokens = tokens;
  a.head = static_cast<const bf16_raw*>(head);
  a.head_n = head_n;
  a.keys = keys;
  a.history = history;
  a.hist_stride = hist_stride;
  a.hist_len = hist_len;
  a.step_ctr = step_ctr;
  a.pos_inc = pos_inc;
  a.bar = bar;
  a.err = err;
  if (hd == 128) return launch_hd<128>(a, grid, stream);
  if (hd == 64) return launch_hd<64>(a, grid, stream);
  return LSA_UNSUPPORTED;
}

#ifdef LSA_PERSIST_STAMPS
extern "C" int lsa_persist_set_stamps(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pstamps), &buf, sizeof(buf)) == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}
#endif
