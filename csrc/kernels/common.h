// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels of llm_sharding_amd.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; workgroups are multiples of 64 threads.
//  * activations are bf16, row-major [rows][cols]; accumulation is fp32.
//  * projection weights are PRE-PACKED once at load time into the MFMA B-fragment order of
//    v_mfma_f32_16x16x32_bf16 ("packed-16x32" layout):
//        Wp[nt][kt][lane][j] = W[nt*16 + (lane & 15)][kt*32 + 8*(lane >> 4) + j]
//    so a wave fetches one 16(n) x 32(k) fragment as ONE fully-contiguous 1 KiB
//    global_load_dwordx4 (16 B/lane) straight into registers - no LDS round trip for the
//    streamed operand (cdna_hip_programming.md §5, 'GEMV / M <= 16' row).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
typedef unsigned short bf16_raw;   // storage type of one bf16 element

#define LSA_WAVE 64
#define LSA_DEVICE __device__ __forceinline__

LSA_DEVICE float bf2f(bf16_raw v) { return __uint_as_float(((unsigned)v) << 16); }

// Round-to-nearest-even fp32 -> bf16 via the native gfx950 conversion (v_cvt_pk_bf16_f32).
LSA_DEVICE bf16_raw f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_raw, b);
}

LSA_DEVICE u32x4_t ld16(const void* p) { return *reinterpret_cast<const u32x4_t*>(p); }
LSA_DEVICE void st16(void* p, u32x4_t v) { *reinterpret_cast<u32x4_t*>(p) = v; }

// Non-temporal 16-byte load for once-read streamed weights (MI355X_MICROARCH.md 'nt-weights').
LSA_DEVICE u32x4_t ld16_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
}

LSA_DEVICE void unpack8(u32x4_t v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

LSA_DEVICE u32x4_t pack8(const float* f) {
  u32x4_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    r[i] = (unsigned)f2bf(f[2 * i]) | ((unsigned)f2bf(f[2 * i + 1]) << 16);
  return r;
}

LSA_DEVICE bf16x8_t as_frag(u32x4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

LSA_DEVICE f32x4_t mfma16(u32x4_t a, u32x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(b), c, 0, 0, 0);
}

template <typename T>
LSA_DEVICE T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over every aligned group of W (8 or 16) lanes, every lane receiving its group's total, on
// DPP lane moves (quad_perm [1,0,3,2] / [2,3,0,1], row_half_mirror, row_mirror): VALU ops
// instead of the ds_bpermute round trips through the LDS crossbar that __shfl_xor compiles to.
template <int CTRL>
LSA_DEVICE float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int W>
LSA_DEVICE float group_sum(float v) {
  static_assert(W == 8 || W == 16, "DPP row groups");
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  v += dpp_mov<0x141>(v);  // row_half_mirror: the other quad of the 8
  if constexpr (W == 16) v += dpp_mov<0x140>(v);  // row_mirror: the other 8 of the 16
  return v;
}

// v of lane (lane ^ OFF), OFF = 8 / 16 / 32, without the LDS crossbar: DPP row_ror:8 (exactly
// lane ^ 8 inside a 16-lane row); v_permlane16_swap / v_permlane32_swap (gfx950) with both
// operands = v leave {even-row, odd-row} (resp. {low-half, high-half}) copies in the pair.
template <int OFF>
LSA_DEVICE float lane_xor(float v) {
  static_assert(OFF == 8 || OFF == 16 || OFF == 32, "lane_xor offsets");
  if constexpr (OFF == 8) {
    return dpp_mov<0x128>(v);
  } else {
    const unsigned u = __builtin_bit_cast(unsigned, v);
    const bool upper = (__lane_id() & OFF) != 0;
    if constexpr (OFF == 16) {
      const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
      return __builtin_bit_cast(float, upper ? r[0] : r[1]);
    } else {
      const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
      return __builtin_bit_cast(float, upper ? r[0] : r[1]);
    }
  }
}

template <typename T>
LSA_DEVICE T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum of squares of 16 values (x0 = columns 0..7, x1 = 8..15) in one fixed rounding order
// (no contraction): the fused RMSNorm's per-64-column partials must be bitwise identical
// whether a residual GEMM's epilogue (gemm_sk) or lsa_row_ss produced them.
LSA_DEVICE float ss16(const float* x0, const float* x1) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) s = __fadd_rn(s, __fadd_rn(__fmul_rn(x0[q], x0[q]), __fmul_rn(x1[q], x1[q])));
  return s;
}

// Orderable 64-bit key for a fused argmax: larger logit wins, ties -> smaller index
// (torch.argmax returns the first maximal index; reference node_worker.py:264).
LSA_DEVICE unsigned long long argmax_key(float v, unsigned idx) {
  unsigned u = __float_as_uint(v);
  unsigned k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)k << 32) | (unsigned long long)(0xffffffffu - idx);
}
LSA_DEVICE unsigned argmax_key_index(unsigned long long key) {
  return 0xffffffffu - (unsigned)(key & 0xffffffffull);
}

// Error codes returned by the extern "C" launchers.
enum LsaStatus { LSA_OK = 0, LSA_BAD_SHAPE = 1, LSA_UNSUPPORTED = 2, LSA_LAUNCH_FAILED = 3 };

#define LSA_CHECK_LAUNCH()                                   \
  do {                                                       \
    if (hipGetLastError() != hipSuccess) return LSA_LAUNCH_FAILED; \
  } while (0)
