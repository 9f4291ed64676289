// Stream-K decode projection for 65..128 rows (and 33..64 with MB = 4): y[M, N] = A[M, K] @ W^T,
// with the fused RMSNorm / RoPE + KV append / SwiGLU / residual / argmax epilogues of epilogue.h.
//
// Why a second kernel beside gemv_coop.hip (profiles/r5_decode128_pmc.md): at 128 rows the coop
// kernel streams the weights at 2.8-4.0 TB/s and parks its waves 32-44 % of their cycles at the
// per-chunk barrier and the register-staged A hand-off, with only two chunks in flight; and its
// (column group x K split) grid fills 172 of the 256 CUs for Llama-2-7B's gate_up (1,376 tiles).
// Here:
//  * exactly one workgroup per CU (grid = 256): the (column group, 64-k chunk) units of the whole
//    projection are dealt out evenly in linear order (stream-K), so every CU streams the same
//    number of weight bytes whatever the tile count; a workgroup's range covers at most a few
//    segments (a tail of one column group, whole groups, a head of the next);
//  * the activations reach LDS by LDS-DMA (global_load_lds_dwordx4) straight into MFMA fragment
//    order - one 1 KiB block per (16 rows, 32 k), lane l's 16 B at l * 16, so every A-fragment
//    read is one lane-linear, conflict-free ds_read_b128 - in a D-slot ring: D - 2 chunks stay in
//    flight across the one s_barrier per chunk (counted vmcnt, static counts);
//  * the weights (packed-16x32, packing.pack_b) go straight to registers (buffer loads, nt) in a
//    D-deep register ring issued with the same chunk, one wave per SIMD owning TNW 16-column
//    tiles (the B operand of TNW x MB MFMAs per A fragment);
//  * a column group split between workgroups is finished by the last contributor to arrive
//    (arrival ticket, write-through fp32 partials, cdna_hip_programming.md §5 'In-launch split-K
//    reduction', sc1 form as gemv_coop.hip), summing the contributors in a fixed order
//    (deterministic, whoever arrives last).
// Reference: the projections are nn.Linear in /root/reference/utils/shard_loader.py:66-74.
#include "epilogue.h"

#include <utility>

// Timing-only ablation builds (scripts/stream_ablate.py; outputs are garbage, only the time
// matters): 1 = no MFMAs / LDS reads in the main loop, 2 = weight loads dropped, 3 = activation
// DMA dropped, 4 = both dropped, 5 = exit after the main loop (no hand-off, no epilogue).
#ifndef LSA_STREAM_ABLATE
#define LSA_STREAM_ABLATE 0
#endif

namespace {

template <int... S, typename F>
LSA_DEVICE bool st_all(std::integer_sequence<int, S...>, F&& f) {
  return (f(std::integral_constant<int, S>{}) && ...);
}

template <int N>
LSA_DEVICE void vm_wait() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

LSA_DEVICE void wg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// One 1 KiB LDS-DMA piece: lane l's 16 B from rsrc + voff + soff to lds + 16 l. (A __device__
// function, not inline in the kernel's lambdas: there the builtin made the host pass drop the
// kernel's launch stub.)
LSA_DEVICE void dma16(__amdgpu_buffer_rsrc_t rs, unsigned char* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// Calls f(slots) with the D ring slots passed through distinct __restrict__ parameters: once
// inlined, every LDS access based on slot s carries its own alias scope, so hipcc's wait
// insertion tracks each slot's LDS-DMA separately and a ds_read of slot s waits only for the DMA
// into slot s - not, as with one undifferentiated LDS array, for every DMA issued before it
// (that inserted vmcnt(0) after each refill and drained the whole ring every step).
template <class F>
LSA_DEVICE void ring_scope(unsigned char* __restrict__ a0, unsigned char* __restrict__ a1, unsigned char* __restrict__ a2,
                           unsigned char* __restrict__ a3, unsigned char* __restrict__ a4, unsigned char* __restrict__ a5,
                           unsigned char* __restrict__ a6, unsigned char* __restrict__ a7, F&& f) {
  unsigned char* const sl[8] = {a0, a1, a2, a3, a4, a5, a6, a7};
  f(sl);
}

// weight loads: nt (aux bit 1), and volatile (bit 31, compiler-only): without it hipcc sinks each
// refill's loads to the end of the unrolled loop body, next to their first use, which leaves
// 0-4 chunks of weights in flight instead of D - 1
constexpr int W_AUX = 2;

// unit u of U (units dealt to W workgroups): workgroup w owns [u0(w), u0(w + 1)), u0(w) = w U / W
LSA_DEVICE int unit0(int w, int U, int W) { return (int)(((long long)w * U) / W); }
LSA_DEVICE int owner(int u, int U, int W) { return (int)((((long long)u + 1) * W + U - 1) / U) - 1; }

// MB: 16-row blocks (rows <= 16 MB); TNW: 16-column tiles per wave; NW: waves (one per SIMD at 4);
// KF: 32-k fragments per chunk; D: ring depth (chunks; D - 2 in flight across a barrier).
template <int MB, int TNW, int NW, int KF, int D, int EPI, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemv_stream_kernel(
    const bf16_raw* __restrict__ x, int ldx, const int* __restrict__ a_rows, const bf16_raw* __restrict__ wp, int M,
    int N, int K, float eps, EpiArgs ep, float* __restrict__ slab, unsigned* __restrict__ counters) {
  constexpr int NTHR = NW * 64;
  constexpr int MR = 16 * MB;
  constexpr int TG = NW * TNW;                 // tiles per column group
  constexpr int KC = 32 * KF;                  // k per chunk
  constexpr int NB = MB * KF;                  // 1 KiB A blocks per chunk
  constexpr int ABUF = NB * 1024;
  constexpr int OPS_A = NB / NW;               // A LDS-DMA instructions per wave per chunk
  constexpr int OPS_W = TNW * KF;              // weight loads per wave per chunk
  constexpr int OPS = OPS_A + OPS_W;
  static_assert(NB % NW == 0, "A blocks must divide over the waves");
  static_assert((D - 2) * OPS <= 63, "counted waits must fit vmcnt");
  static_assert(D >= 3, "ring depth");
  constexpr int RS = 20;                       // epilogue staging row stride (floats)
  constexpr int RH = MR < 64 ? MR : 64;        // rows per epilogue pass
  constexpr int EPW = 2 * RH * RS;             // floats per wave in an epilogue pass (<= 2 tiles)
  constexpr int SMEM = (D * ABUF > NW * EPW * 4) ? D * ABUF : NW * EPW * 4;
  constexpr int FR = TG * MB * 256;            // floats of one fp32 partial (fragment-native)
  static_assert(EPI != EPI_SWIGLU || TNW % 2 == 0, "SwiGLU: gate / up tile pairs inside one wave");
  static_assert(EPI != EPI_PARTIAL, "no EPI_PARTIAL");

  // ALL of the kernel's LDS is this one array (cdna_hip_programming.md, 'Projection GEMM at M = 256'
  // item 4(a): a second __shared__ object made hipcc wait vmcnt(0) before the first ds_read of
  // every step, draining the DMA ring): the ring / epilogue staging area, then the small arrays
  constexpr int OFF_KEY = SMEM, OFF_SSB = OFF_KEY + MR * 8, OFF_SSP = OFF_SSB + NB * 16 * 4,
                OFF_SS = OFF_SSP + MR * 4, OFF_LAST = OFF_SS + MR * 4, SMEM_ALL = OFF_LAST + 16;
  static_assert(SMEM_ALL <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM_ALL];
  unsigned long long* s_key = reinterpret_cast<unsigned long long*>(smem + OFF_KEY);
  float (*s_ssb)[16] = reinterpret_cast<float (*)[16]>(smem + OFF_SSB);  // per A block row sums of squares
  float* s_ssp = reinterpret_cast<float*>(smem + OFF_SSP);               // this segment's row sums of squares
  float* s_ss = reinterpret_cast<float*>(smem + OFF_SS);
  int& s_last = *reinterpret_cast<int*>(smem + OFF_LAST);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int KT = K >> 5;
  const int nch = K / KC;                       // chunks per column group
  const int G = N / 16 / TG;
  const int U = G * nch, WG = gridDim.x, wg = blockIdx.x;
  const int u_beg = unit0(wg, U, WG), u_end = unit0(wg + 1, U, WG);

  // ---- per-lane A sources: block b = w * OPS_A + i -> (kf, rb) = (b / MB, b % MB); lane l loads
  // row rb*16 + (l & 15), k kf*32 + 8 (l >> 4) .. + 8 of every chunk (rows >= M read row 0: valid
  // memory, never stored; their sum of squares is never used)
  int avoff[OPS_A];
#pragma unroll
  for (int i = 0; i < OPS_A; ++i) {
    const int b = w * OPS_A + i, kf = b / MB, rb = b % MB;
    const int r = rb * 16 + (lane & 15);
    const int rr = r < M ? (a_rows ? a_rows[r] : r) : 0;
    avoff[i] = (rr * ldx + kf * 32 + 8 * (lane >> 4)) * 2;
  }
  // every step issues the same loads (static counted waits, and hipcc's own waits for the weight
  // registers stay counted): a step past the segment's end re-loads the segment's last chunk (an
  // L2 hit) into the free slot. Not a zero-record descriptor: a load its range check drops can
  // retire before older loads, and a counted vmcnt then passed with a chunk still in flight (a
  // wrong 16 x 16 block at 2 waves per SIMD, tests/test_gemv_stream_gpu.py)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0x7fffffff, 0x00020000);
  // ablation builds only: descriptors with zero records (every load through them dropped)
  const __amdgpu_buffer_rsrc_t xr0 = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr0 = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc((void*)slab, (short)0, 0x7fffffff, 0x00020000);
  const int lane16 = lane * 16;

  u32x4_t wreg[D][KF][TNW];
  f32x4_t acc[MB][TNW];
  float ssl[OPS_A];

  if (EPI == EPI_ARGMAX)
    for (int r = tid; r < MR; r += NTHR) s_key[r] = 0ull;

  for (int u = u_beg; u < u_end;) {
    const int g = u / nch, ca = u - g * nch;
    const int cb = (u_end - g * nch) < nch ? (u_end - g * nch) : nch;
    const int n = cb - ca;
    const int nt0 = g * TG + w * TNW;          // this wave's first tile
#pragma unroll
    for (int rb = 0; rb < MB; ++rb)
#pragma unroll
      for (int t = 0; t < TNW; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < OPS_A; ++i) ssl[i] = 0.f;

    static_assert(D <= 8, "ring_scope passes 8 slots");
    ring_scope(smem, smem + ABUF * (D > 1), smem + ABUF * 2 * (D > 2), smem + ABUF * 3 * (D > 3),
               smem + ABUF * 4 * (D > 4), smem + ABUF * 5 * (D > 5), smem + ABUF * 6 * (D > 6),
               smem + ABUF * 7 * (D > 7), [&](unsigned char* const* sl) {
      auto issue = [&](int c_in, auto slot_c) {  // chunk c (group-relative) into ring slot S
        constexpr int S = decltype(slot_c)::value;
        const int c = c_in < cb ? c_in : cb - 1;
        const bool a_live = LSA_STREAM_ABLATE != 3 && LSA_STREAM_ABLATE != 4;
        const bool w_live = LSA_STREAM_ABLATE != 2 && LSA_STREAM_ABLATE != 4;
        const __amdgpu_buffer_rsrc_t xs = a_live ? xr : xr0, ws = w_live ? wr : wr0;
        unsigned char* dst = sl[S];
#pragma unroll
        for (int i = 0; i < OPS_A; ++i)
          dma16(xs, dst + (w * OPS_A + i) * 1024, avoff[i], c * KC * 2);
#pragma unroll
        for (int f = 0; f < KF; ++f)
#pragma unroll
          for (int t = 0; t < TNW; ++t)
            wreg[S][f][t] = __builtin_amdgcn_raw_buffer_load_b128(ws, lane16, ((nt0 + t) * KT + c * KF + f) * 1024, W_AUX);
      };
      auto compute = [&](auto slot_c) {
        constexpr int S = decltype(slot_c)::value;
        const unsigned char* src = sl[S] + lane16;
        if (NORM) {  // sum of squares of the A blocks this wave staged (fixed block per ssl slot)
#pragma unroll
          for (int i = 0; i < OPS_A; ++i) {
            float v[8];
            unpack8(*reinterpret_cast<const u32x4_t*>(src + (w * OPS_A + i) * 1024), v);
#pragma unroll
            for (int j = 0; j < 8; ++j) ssl[i] = __builtin_fmaf(v[j], v[j], ssl[i]);
          }
        }
#pragma unroll
        for (int f = 0; f < KF; ++f) {
          u32x4_t af[MB];
#pragma unroll
          for (int rb = 0; rb < MB; ++rb) af[rb] = *reinterpret_cast<const u32x4_t*>(src + (f * MB + rb) * 1024);
#pragma unroll
          for (int rb = 0; rb < MB; ++rb)
#pragma unroll
            for (int t = 0; t < TNW; ++t) acc[rb][t] = mfma16(af[rb], wreg[S][f][t], acc[rb][t]);
        }
      };
      // prologue: chunks 0 .. D - 2 of the segment into slots 0 ..
      st_all(std::make_integer_sequence<int, D - 1>{}, [&](auto s) {
        issue(ca + decltype(s)::value, s);
        __builtin_amdgcn_sched_barrier(0);
        return true;
      });
      // step i (slot i % D): wait for chunk i (D - 2 later chunks stay in flight), barrier (its DMA
      // from every wave has landed and every wave is done with slot (i - 1) % D), refill that slot
      // with chunk i + D - 1, compute chunk i
      // The full groups of D steps run as ONE basic block per loop iteration (no early exit inside):
      // with an exit test between steps, hipcc moved every refill's weight loads down to the last
      // step of the unrolled body, next to their first use. The < D remaining steps follow with
      // exits; the chunks they issue are all past the segment's end (dropped loads).
      int i = 0;
      auto step = [&](auto s) {
        constexpr int S = decltype(s)::value;
        vm_wait<(D - 2) * OPS>();
        wg_barrier();
        issue(ca + i + D - 1, std::integral_constant<int, (S + D - 1) % D>{});
        __builtin_amdgcn_sched_barrier(0);  // the refill stays ahead of this chunk's MFMAs
        if constexpr (LSA_STREAM_ABLATE != 1) compute(s);
        __builtin_amdgcn_sched_barrier(0);
        ++i;
        return true;
      };
      for (int it = n / D; it > 0; --it) st_all(std::make_integer_sequence<int, D>{}, step);
      st_all(std::make_integer_sequence<int, D>{}, [&](auto s) { return i < n && step(s); });
    });
    vm_wait<0>();  // the dropped loads of the last steps
    wg_barrier();  // every wave is done with the ring: it becomes the epilogue staging area

    // ---- this segment's row sums of squares (NORM): block b's lanes l, l^16, l^32, l^48 hold one
    // row; the KF blocks of a row block are added in k order
    if (NORM) {
#pragma unroll
      for (int i = 0; i < OPS_A; ++i) {
        float v = ssl[i];
        v += lane_xor<16>(v);
        v += lane_xor<32>(v);
        if (lane < 16) s_ssb[w * OPS_A + i][lane] = v;
      }
      __syncthreads();
      for (int r = tid; r < MR; r += NTHR) {
        float t2 = 0.f;
#pragma unroll
        for (int f = 0; f < KF; ++f) t2 += s_ssb[f * MB + r / 16][r % 16];
        s_ssp[r] = t2;
      }
    }

    if constexpr (LSA_STREAM_ABLATE == 5) {
      float t = 0.f;
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int q = 0; q < TNW; ++q) t += acc[rb][q][0];
      if (t == 1.2345f) ep.out[tid] = 0;  // keep the loop live
      u = g * nch + cb;
      continue;
    }
    const bool whole = ca == 0 && cb == nch;
    bool finish = whole;
    if (!whole) {
      // ---- split group: store this contributor's partial (write-through), take a ticket
      const int slot = 2 * wg + (u == u_beg ? 0 : 1);
#pragma unroll
      for (int rb = 0; rb < MB; ++rb)
#pragma unroll
        for (int t = 0; t < TNW; ++t)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[rb][t]), sr,
                                                 ((((w * TNW + t) * MB + rb) * 64 + lane) * 4) * 4, slot * FR * 4, 16);
      __syncthreads();  // s_ssp written
      if (NORM)
        for (int r = tid; r < MR; r += NTHR)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s_ssp[r]), sr, (slot * MR + r) * 4,
                                                2 * WG * FR * 4, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int wf = owner(g * nch, U, WG), wl = owner(g * nch + nch - 1, U, WG);
        const unsigned old = __hip_atomic_fetch_add(&counters[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (unsigned)(wl - wf);
      }
      __syncthreads();
      finish = s_last != 0;
      if (finish) {
        // last arriver: the group's contributors wf .. wl summed in that order (its own partial
        // included, read back like the others), CQ contributors x RBQ row blocks of loads in flight
        // per round trip
        const int wf = owner(g * nch, U, WG), wl = owner(g * nch + nch - 1, U, WG);
#pragma unroll
        for (int rb = 0; rb < MB; ++rb)
#pragma unroll
          for (int t = 0; t < TNW; ++t) acc[rb][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        auto slot_of = [&](int ww) { return 2 * ww + (unit0(ww, U, WG) >= g * nch ? 0 : 1); };
        constexpr int RBQ = MB / 2 > 0 ? MB / 2 : 1;
        constexpr int CQ = 16 / (RBQ * TNW) > 1 ? 16 / (RBQ * TNW) : 1;
        for (int j0 = wf; j0 <= wl; j0 += CQ) {
#pragma unroll
          for (int h0 = 0; h0 < MB; h0 += RBQ) {
            f32x4_t v[CQ][RBQ][TNW];
#pragma unroll
            for (int q = 0; q < CQ; ++q) {
              const int ww = j0 + q <= wl ? j0 + q : wl;
              const int so = slot_of(ww) * FR * 4;
#pragma unroll
              for (int rb = 0; rb < RBQ; ++rb)
#pragma unroll
                for (int t = 0; t < TNW; ++t)
                  v[q][rb][t] = __builtin_bit_cast(
                      f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                   sr, ((((w * TNW + t) * MB + h0 + rb) * 64 + lane) * 4) * 4, so, 16));
            }
#pragma unroll
            for (int q = 0; q < CQ; ++q)
              if (j0 + q <= wl)
#pragma unroll
                for (int rb = 0; rb < RBQ; ++rb)
#pragma unroll
                  for (int t = 0; t < TNW; ++t) acc[h0 + rb][t] += v[q][rb][t];
          }
        }
        if (NORM) {
          for (int r = tid; r < MR; r += NTHR) {
            float t2 = 0.f;
            for (int ww = wf; ww <= wl; ++ww)
              t2 += __uint_as_float(
                  __builtin_amdgcn_raw_buffer_load_b32(sr, (slot_of(ww) * MR + r) * 4, 2 * WG * FR * 4, 16));
            s_ss[r] = t2;
          }
        }
        if (tid == 0) __hip_atomic_store(&counters[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (NORM) {
      __syncthreads();
      for (int r = tid; r < MR; r += NTHR) s_ss[r] = s_ssp[r];
    }

    if (finish) {
      __syncthreads();  // s_ss complete
      // ---- epilogue: per wave, tiles in pairs (SwiGLU: gate 2p / up 2p + 1), rows in passes of RH;
      // the accumulators go through a wave-private LDS image, then lane l finishes row l of the pass
      float* img = reinterpret_cast<float*>(smem) + w * EPW;
      constexpr int TP = TNW >= 2 ? 2 : 1;
#pragma unroll
      for (int p = 0; p < TNW / TP; ++p) {
#pragma unroll
        for (int h = 0; h < MR / RH; ++h) {
#pragma unroll
          for (int q = 0; q < TP; ++q)
#pragma unroll
            for (int rb = 0; rb < RH / 16; ++rb)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                img[(q * RH + rb * 16 + (lane >> 4) * 4 + r) * RS + (lane & 15)] = acc[h * (RH / 16) + rb][p * TP + q][r];
          __syncthreads();
          const int mm = h * RH + lane;
          if (lane < RH && mm < M) {
            const float rs = NORM ? rsqrtf(s_ss[mm] / (float)K + eps) : 1.f;
            float v[TP][16];
#pragma unroll
            for (int q = 0; q < TP; ++q)
#pragma unroll
              for (int c4 = 0; c4 < 4; ++c4) {
                const f32x4_t x4 = *reinterpret_cast<const f32x4_t*>(img + (q * RH + lane) * RS + 4 * c4);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[q][4 * c4 + j] = x4[j] * rs;
              }
            const int tile0 = nt0 + p * TP;
            if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
              for (int j = 0; j < 16; ++j) v[0][j] = silu(v[0][j]) * v[TP - 1][j];
              bf16_raw* o = ep.out + (size_t)mm * ep.ldo + (tile0 / 2) * 16;
              st16(o, pack8(v[0]));
              st16(o + 8, pack8(v[0] + 8));
            } else if constexpr (EPI == EPI_ARGMAX) {
              unsigned long long key = 0ull;
#pragma unroll
              for (int q = 0; q < TP; ++q) {
                epi_bias16(ep, (tile0 + q) * 16, v[q]);
                const unsigned long long kq = argmax_key16(v[q], (unsigned)((tile0 + q) * 16 + ep.col_offset));
                key = kq > key ? kq : key;
              }
              atomicMax(&s_key[mm], key);
            } else {
#pragma unroll
              for (int q = 0; q < TP; ++q) epi_row16<EPI>(ep, mm, (tile0 + q) * 16, v[q]);
            }
          }
          __syncthreads();
        }
      }
    }
    u = g * nch + cb;
    __syncthreads();  // the ring / staging area and s_ssp are reused by the next segment
  }
  if (EPI == EPI_ARGMAX) {
    __syncthreads();
    for (int r = tid; r < M; r += NTHR)
      if (s_key[r]) atomicMax(&ep.keys[r], s_key[r]);
  }
}

template <int MB, int TNW, int NW, int KF, int D, int EPI>
int launch(bool norm, const bf16_raw* x, int ldx, const int* a_rows, const bf16_raw* wp, int M, int N, int K, float eps,
           const EpiArgs& ep, float* slab, unsigned* cnt, int grid, hipStream_t s) {
  if (norm)
    gemv_stream_kernel<MB, TNW, NW, KF, D, EPI, true><<<grid, NW * 64, 0, s>>>(x, ldx, a_rows, wp, M, N, K, eps, ep, slab, cnt);
  else
    gemv_stream_kernel<MB, TNW, NW, KF, D, EPI, false><<<grid, NW * 64, 0, s>>>(x, ldx, a_rows, wp, M, N, K, eps, ep, slab, cnt);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

// (mb, tnw, nw, kf, d) instantiated; keep ops/packing.py STREAM_CONFIGS in sync
#define LSA_STREAM_CONFIGS(X) \
  X(8, 2, 4, 2, 6) X(8, 1, 4, 2, 6) X(8, 1, 8, 2, 6) X(8, 2, 8, 2, 4) X(8, 1, 8, 2, 8)

template <int EPI>
int dispatch(int mb, int tnw, int nw, int kf, int d, bool norm, const bf16_raw* x, int ldx, const int* a_rows,
             const bf16_raw* wp, int M, int N, int K, float eps, const EpiArgs& ep, float* slab, unsigned* cnt, int grid,
             hipStream_t s) {
#define LSA_C(B, T, W, F, DD)                                                                           \
  if constexpr (EPI != EPI_SWIGLU || T % 2 == 0)                                                        \
    if (mb == B && tnw == T && nw == W && kf == F && d == DD)                                           \
      return launch<B, T, W, F, DD, EPI>(norm, x, ldx, a_rows, wp, M, N, K, eps, ep, slab, cnt, grid, s);
  LSA_STREAM_CONFIGS(LSA_C)
#undef LSA_C
  return LSA_UNSUPPORTED;
}

}  // namespace

// grid: workgroups (one per CU: 256 on MI355X; every workgroup needs >= 1 chunk). Workspace:
// slab >= 2 * grid * (tnw * nw * 16 * 16 * mb + 16 * mb) floats; counters: N / 16 / (tnw * nw)
// zero-initialised uint32 (each reset by the group's last contributor, replay-safe in hipGraphs).
extern "C" int lsa_gemv_stream(const void* x, int ldx, const int* a_rows, const void* wp, int M, int N, int K, int norm,
                               float eps, int epi, const EpiArgs* ep, int tnw, int nw, int kf, int depth, int grid,
                               float* slab, unsigned* counters, hipStream_t stream) {
  const int mb = M <= 64 ? 4 : 8;
  if (M < 1 || M > 128 || kf < 1 || K % (32 * kf) || ldx < K || grid < 1 || !slab || !counters) return LSA_BAD_SHAPE;
  const int tg = nw * tnw;
  if (N % (16 * tg)) return LSA_BAD_SHAPE;
  if ((long long)(N / 16 / tg) * (K / (32 * kf)) < grid) return LSA_BAD_SHAPE;  // >= 1 chunk per workgroup
  if (epi == EPI_SWIGLU && tnw % 2) return LSA_BAD_SHAPE;
  const bf16_raw* xx = static_cast<const bf16_raw*>(x);
  const bf16_raw* w = static_cast<const bf16_raw*>(wp);
  const bool n = norm != 0;
#define LSA_D(E) dispatch<E>(mb, tnw, nw, kf, depth, n, xx, ldx, a_rows, w, M, N, K, eps, *ep, slab, counters, grid, stream)
  switch (epi) {
    case EPI_STORE: return LSA_D(EPI_STORE);
    case EPI_RESID: return LSA_D(EPI_RESID);
    case EPI_SWIGLU: return LSA_D(EPI_SWIGLU);
    case EPI_QKV: return LSA_D(EPI_QKV);
    case EPI_ARGMAX: return LSA_D(EPI_ARGMAX);
    default: return LSA_UNSUPPORTED;
  }
#undef LSA_D
}
