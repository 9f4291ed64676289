// Probe (never part of the product library; built into build/probes/ by
// scripts/probes/build_chain_probe.sh): does ONE persistent launch with a run-ahead weight loader
// beat separate launches for a batch-1 decode chain on MI355X?
//
// The chain is the weight-streaming part of a Llama-2-7B layer at batch 1, attention and norms
// left out: y0 = W0 x0 (12288 x 4096, "qkv"), y1 = W1 y0[:4096] (4096 x 4096, "o"),
// y2 = W2 y1 (22016 x 4096, "gate_up"), y3 = W3 y2[:11008] (4096 x 11008, "down"); bf16 weights,
// row-major [N][K], fp32 accumulation, bf16 outputs. The baseline is the library's tuned decode
// GEMV (gemv.hip) launched once per op (scripts/probes/chain_probe.py).
//
// Persistent form (MI355X_MICROARCH.md 'engine-vs-launches', 'prefetch-credit', granule rows):
//  * 256 workgroups, one per CU; workgroup g owns rows [g R_p, (g+1) R_p) of every op (R_p = N_p / 256),
//    a contiguous R_p x K_p slice of W_p.
//  * wave 0 is the LOADER: it streams the workgroup's slices of all four ops, in op order, through an
//    NS-slot LDS ring of 16 KiB slots by LDS-DMA (global_load_lds, non-temporal), keeping D slots in
//    flight (counted vmcnt) and publishing each landed slot with a generation word in LDS. It never
//    waits on data dependencies, only on a slot being FREE, so it runs ahead across every op
//    boundary: the next op's weights stream while the consumers wait for its input.
//  * waves 1..4 are CONSUMERS: per op they gather the input vector from the previous op's output
//    granules (8 bytes = 2 bf16 + a 32-bit tag written by ONE write-through store; tag = epoch * 4 +
//    op + 1, so no flag, counter or grid barrier exists), then reduce every published slot: lane l
//    takes 32 consecutive weights of one row, dots them with x (fp32 FMAs) and adds the
//    partial into an LDS row accumulator; each wave frees the slot after its reads retired.
//  * every spin is bounded (SPIN_MAX polls with s_sleep): a missing producer sets *err and the
//    workgroup runs to its end, so the grid always drains.
// Row accumulation: a wave-level reduction, then LDS float atomics (order not fixed): a probe, not
// bit-reproducible.
#include "common.h"

namespace {

constexpr int P = 4;
constexpr int NCW = 4;                  // consumer waves
constexpr int NLW = 4;                  // loader waves (each issues PIECES / NLW of every slot)
constexpr int NTHR = (NCW + NLW) * 64;
constexpr int SLOT = 16384;             // bytes per ring slot
constexpr int PIECES = SLOT / 1024;     // 1 KiB DMA pieces per slot (64 lanes x 16 B)
constexpr int D = 5;                    // slots the loaders keep in flight
constexpr int NS = D + 3;               // ring slots (>= in flight + 3, 'ring-gemm')
constexpr int PPL = PIECES / NLW;       // pieces per loader wave and slot
constexpr int MAXK = 11008;
constexpr int MAXR = 96;
constexpr unsigned SPIN_MAX = 1u << 21;

struct ChainArgs {
  const bf16_raw* w[P];
  int N[P], K[P];
  const bf16_raw* x0;
  unsigned long long* gran[P];  // op p's output as N_p / 2 granules {2 x bf16 | tag << 32}
  unsigned* err;  // [0] flags, [1] staged-weight mismatches, [2] staged-x mismatches (check)
  unsigned epoch;
  int check;
};

LSA_DEVICE unsigned lds_load(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }

__global__ __launch_bounds__(NTHR) void chain_kernel(ChainArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[NS * SLOT];
  __shared__ __attribute__((aligned(16))) bf16_raw xs[MAXK];
  __shared__ float acc[MAXR];
  __shared__ unsigned full_gen[NS], free_cnt[NS], cbar;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (tid < NS) {
    full_gen[tid] = 0;
    free_cnt[tid] = 0;
  }
  if (tid == 0) cbar = 0;
  for (int i = tid; i < MAXR; i += NTHR) acc[i] = 0.f;
  __syncthreads();  // the only whole-workgroup barrier
  const int g = blockIdx.x, G = gridDim.x;

  if (w < NLW) {
    // ------------------------------------------------------------------ loader
    int s = 0;
    auto publish = [&](int sp) {  // this wave's part of slot sp landed (caller waited for it)
      if (lane == 0) __hip_atomic_fetch_add(&full_gen[sp % NS], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    for (int p = 0; p < P; ++p) {
      const int R = a.N[p] / G, K = a.K[p];
      const long long bytes = (long long)R * K * 2;
      const unsigned char* base = reinterpret_cast<const unsigned char*>(a.w[p] + (size_t)g * R * K);
      const int nsl = (int)((bytes + SLOT - 1) / SLOT);
      for (int j = 0; j < nsl; ++j, ++s) {
        const int i = s % NS;
        const unsigned need = (unsigned)(NCW * (s / NS));
        unsigned spins = 0;
        while (lds_load(&free_cnt[i]) < need) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_MAX) { if (lane == 0) atomicOr(a.err, 1u); break; }
        }
#pragma unroll
        for (int q = w * PPL; q < (w + 1) * PPL; ++q) {
          long long off = (long long)j * SLOT + q * 1024 + lane * 16;
          if (off >= bytes) off = 0;  // tail of the last slot: any valid address (never consumed)
          __builtin_amdgcn_global_load_lds(base + off, (__attribute__((address_space(3))) void*)(ring + i * SLOT + q * 1024),
                                           16, 0, 2 /* nt */);
        }
        if (s >= D - 1) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PPL * (D - 1)) : "memory");
          publish(s - (D - 1));
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int sp = (s - (D - 1) > 0 ? s - (D - 1) : 0); sp < s; ++sp) publish(sp);  // the last D-1 slots
    return;
  }

  // -------------------------------------------------------------------- consumers
  const int cl = tid - NLW * 64;  // 0 .. NCW*64-1
  unsigned nbar = 0;
  auto cons_barrier = [&]() {  // the NCW consumer waves only (the loader never joins)
    ++nbar;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(&cbar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned spins = 0;
    while (lds_load(&cbar) < NCW * nbar) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > SPIN_MAX) { if (lane == 0) atomicOr(a.err, 2u); break; }
    }
  };
  const __amdgpu_buffer_rsrc_t xr0 = __builtin_amdgcn_make_buffer_rsrc((void*)a.x0, (short)0, 0x7fffffff, 0x00020000);
  int s = 0;
  for (int p = 0; p < P; ++p) {
    const int R = a.N[p] / G, K = a.K[p];
    const long long nel = (long long)R * K;
    const int nsl = (int)((nel * 2 + SLOT - 1) / SLOT);
    // 1. the input vector into LDS
    if (p == 0) {
      for (int k = cl * 8; k < K; k += NCW * 64 * 8)
        *reinterpret_cast<u32x4_t*>(xs + k) = __builtin_amdgcn_raw_buffer_load_b128(xr0, k * 2, 0, 0);
    } else {
      const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc((void*)a.gran[p - 1], (short)0, 0x7fffffff, 0x00020000);
      const unsigned want = a.epoch * P + (unsigned)p;  // tag of op p-1
      // every granule of this lane requested in one pass (independent loads in flight together),
      // then checked; a pass with any tag missing is repeated (bounded)
      constexpr int GPL = (MAXK / 2 + NCW * 64 - 1) / (NCW * 64);
      unsigned spins = 0;
      for (;;) {
        u32x2_t v[GPL];
#pragma unroll
        for (int t = 0; t < GPL; ++t) {
          const int gi = cl + t * NCW * 64;
          v[t] = gi < K / 2 ? __builtin_amdgcn_raw_buffer_load_b64(gr, gi * 8, 0, 16 /* sc1 */) : u32x2_t{0u, want};
        }
        bool all = true;
#pragma unroll
        for (int t = 0; t < GPL; ++t) {
          const int gi = cl + t * NCW * 64;
          if (v[t][1] == want) {
            if (gi < K / 2) *reinterpret_cast<unsigned*>(xs + 2 * gi) = v[t][0];
          } else {
            all = false;
          }
        }
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_MAX) { atomicOr(a.err, 4u); break; }
      }
    }
    cons_barrier();
    // 2. reduce the op's slots
    for (int j = 0; j < nsl; ++j, ++s) {
      const int i = s % NS;
      const unsigned gen = (unsigned)(NLW * (s / NS + 1));  // every loader wave's part landed
      unsigned spins = 0;
      while (lds_load(&full_gen[i]) < gen) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_MAX) { if (lane == 0) atomicOr(a.err, 8u); break; }
      }
      const long long e0 = (long long)j * (SLOT / 2) + cl * 32;
      float d = 0.f;
      int row = -1;
      if (e0 < nel) {
        row = (int)(e0 / K);
        const int col = (int)(e0 - (long long)row * K);
        const u32x4_t* wv = reinterpret_cast<const u32x4_t*>(ring + i * SLOT + cl * 64);
        const u32x4_t* xv = reinterpret_cast<const u32x4_t*>(xs + col);
        if (a.check) {  // debug: the staged bytes against the same bytes read from memory
          const u32x4_t* gv = reinterpret_cast<const u32x4_t*>(a.w[p] + (size_t)g * R * K + e0);
          bool bad = false;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const u32x4_t x1 = wv[q], x2 = gv[q];
            bad |= x1[0] != x2[0] || x1[1] != x2[1] || x1[2] != x2[2] || x1[3] != x2[3];
          }
          if (bad) atomicAdd(a.err + 1, 1u);
          if (p == 0) {
            const u32x4_t* gx = reinterpret_cast<const u32x4_t*>(a.x0 + col);
            bool badx = false;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const u32x4_t x1 = xv[q], x2 = gx[q];
              badx |= x1[0] != x2[0] || x1[1] != x2[1] || x1[2] != x2[2] || x1[3] != x2[3];
            }
            if (badx) atomicAdd(a.err + 2, 1u);
          }
        }
        // fp32 FMAs on unpacked bf16 (hipcc 7.2 folded the four v_dot2c_f32_bf16 of a 16-B chunk onto
        // its first dword pair - the first build of this probe computed wrong rows)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float wf[8], xf[8];
          unpack8(wv[q], wf);
          unpack8(xv[q], xf);
#pragma unroll
          for (int e = 0; e < 8; ++e) d = __builtin_fmaf(wf[e], xf[e], d);
        }
      }
      // wave-level reduction first (a 4 KiB wave chunk spans at most two consecutive rows: rows are
      // >= 8 KiB), then one LDS atomic per row and wave instead of 64 on one address
      const int row0 = __builtin_amdgcn_readfirstlane(row);
      const bool hasb = __builtin_amdgcn_ballot_w64(row0 >= 0 && row == row0 + 1) != 0;
      float da = row == row0 ? d : 0.f, db = (row0 >= 0 && row == row0 + 1) ? d : 0.f;
      da = group_sum<16>(da);
      da += lane_xor<16>(da);
      da += lane_xor<32>(da);
      db = group_sum<16>(db);
      db += lane_xor<16>(db);
      db += lane_xor<32>(db);
      if (row0 >= 0 && lane == 0) __hip_atomic_fetch_add(&acc[row0], da, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (hasb && lane == 0) __hip_atomic_fetch_add(&acc[row0 + 1], db, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's ring reads retired
      if (lane == 0) __hip_atomic_fetch_add(&free_cnt[i], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    cons_barrier();  // every partial added
    // 3. publish the rows as granules (one 8-byte write-through store each), reset the accumulators
    if (cl < R / 2) {
      const unsigned data = (unsigned)f2bf(acc[2 * cl]) | ((unsigned)f2bf(acc[2 * cl + 1]) << 16);
      const u32x2_t v = {data, a.epoch * P + (unsigned)p + 1};
      const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc((void*)a.gran[p], (short)0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b64(v, orr, (g * (R / 2) + cl) * 8, 0, 16 /* sc1 */);
    }
    cons_barrier();
    if (cl < MAXR) acc[cl] = 0.f;
  }
}

}  // namespace

extern "C" int lsa_chain_probe(const void* const* w, const int* N, const int* K, const void* x0,
                               unsigned long long* const* gran, unsigned* err, unsigned epoch, int check,
                               hipStream_t stream) {
  ChainArgs a;
  for (int p = 0; p < P; ++p) {
    if (N[p] % 256 || N[p] / 256 > MAXR || (N[p] / 256) % 2 || K[p] % 32 || K[p] > MAXK) return LSA_BAD_SHAPE;
    if (p > 0 && K[p] > N[p - 1]) return LSA_BAD_SHAPE;
    a.w[p] = static_cast<const bf16_raw*>(w[p]);
    a.N[p] = N[p];
    a.K[p] = K[p];
    a.gran[p] = gran[p];
  }
  a.x0 = static_cast<const bf16_raw*>(x0);
  a.err = err;
  a.epoch = epoch;
  a.check = check;
  chain_kernel<<<256, NTHR, 0, stream>>>(a);
  return hipGetLastError() == hipSuccess ? LSA_OK : LSA_LAUNCH_FAILED;
}
