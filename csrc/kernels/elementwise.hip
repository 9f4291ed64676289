// Small bandwidth-bound kernels of the stage forward, all vectorised 16 B/lane
// (cdna_hip_programming.md Guideline 13):
//   lsa_embed        nn.Embedding row gather (reference node_worker.py:215,302)
//   lsa_rmsnorm      standalone RMSNorm (prefill path; decode fuses it into the GEMV)
//   lsa_resid_rmsnorm_partials  residual add of split-K GEMM partials + the next RMSNorm
//   lsa_layernorm    LayerNorm with bias (GPT-2 ln_1 / ln_2 / ln_f), optionally fused with the
//                    learned absolute position embedding add (x += wpe[pos], written back)
//   lsa_argmax_finalize  decode the fused-argmax keys -> token ids, reset the keys, append to
//                    the device-side history and advance the per-row positions. This keeps
//                    the whole autoregressive step on the device (no .item() host sync per
//                    token as in node_worker.py:287) so it can be captured in a hipGraph.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ ids,
                                                    const bf16_raw* __restrict__ table, int H,
                                                    bf16_raw* __restrict__ out, int ldo) {
  const int row = blockIdx.x;
  const int id = ids[row];
  const bf16_raw* src = table + (size_t)id * H;
  bf16_raw* dst = out + (size_t)row * ldo;
  for (int c = threadIdx.x; c < (H >> 3); c += blockDim.x) st16(dst + c * 8, ld16(src + c * 8));
}

__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_raw* __restrict__ x, int ldx,
                                                      const bf16_raw* __restrict__ w, int H,
                                                      float eps, bf16_raw* __restrict__ out,
                                                      int ldo) {
  __shared__ float s_part[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_raw* xr = x + (size_t)row * ldx;
  float s = 0.f;
  for (int c = tid; c < (H >> 3); c += 256) {
    float f[8];
    unpack8(ld16(xr + c * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[j] * f[j];
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) s_part[tid >> 6] = s;
  __syncthreads();
  const float rs = rsqrtf((s_part[0] + s_part[1] + s_part[2] + s_part[3]) / (float)H + eps);
  bf16_raw* orow = out + (size_t)row * ldo;
  for (int c = tid; c < (H >> 3); c += 256) {
    float f[8], g[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
    unpack8(ld16(xr + c * 8), f);
    if (w) unpack8(ld16(w + c * 8), g);  // w == nullptr: weight folded into the next GEMM
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = f[j] * rs * g[j];
    st16(orow + c * 8, pack8(f));
  }
}

// Register-resident RMSNorm for H = 2048 * NC (Llama-2-7B / 70B: NC = 2 / 4; other widths take
// rmsnorm_kernel), used by the engine's standalone norms of >128-row forwards: every lane issues
// its NC 16-B row loads (and the weight's) before the first use, so a row costs ONE memory round
// trip and is not re-read for the scaling pass. Same per-lane accumulation order as rmsnorm_kernel.
template <int NC>
__global__ __launch_bounds__(256) void rmsnorm_reg_kernel(const bf16_raw* __restrict__ x, int ldx,
                                                          const bf16_raw* __restrict__ w,
                                                          float eps, bf16_raw* __restrict__ out,
                                                          int ldo) {
  constexpr int H = 2048 * NC;
  __shared__ float s_part[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_raw* xr = x + (size_t)row * ldx;
  u32x4_t v[NC], wv[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) v[j] = ld16(xr + (tid + j * 256) * 8);
  if (w) {
#pragma unroll
    for (int j = 0; j < NC; ++j) wv[j] = ld16(w + (tid + j * 256) * 8);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    float f[8];
    unpack8(v[j], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += f[k] * f[k];
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) s_part[tid >> 6] = s;
  __syncthreads();
  const float rs = rsqrtf((s_part[0] + s_part[1] + s_part[2] + s_part[3]) / (float)H + eps);
  bf16_raw* orow = out + (size_t)row * ldo;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    float f[8], g[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
    unpack8(v[j], f);
    if (w) unpack8(wv[j], g);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = f[k] * rs * g[k];
    st16(orow + (tid + j * 256) * 8, pack8(f));
  }
}

// Residual add of split-K GEMM partials fused with the next RMSNorm (gemm_sk EPI_PARTIAL):
//   h[row] = bf16(h[row] + (P[0][row] + ... + P[S-1][row]))   (fixed order: reproducible)
//   out[row] = rmsnorm(h[row]) * w                              (skipped when out == nullptr)
// The o / down projections of a >128-row forward end in a residual add that is always followed
// by an RMSNorm (post-attention norm, next layer's input norm or the final norm): summing their
// K-split partials here replaces the GEMM's slab + ticket + last-arriver fixup tail. H = 2048 * NC,
// register-resident: every lane issues all its loads before the first use.
template <int NC>
__global__ __launch_bounds__(256) void resid_norm_partials_kernel(bf16_raw* __restrict__ h, int ldh,
                                                                  const float* __restrict__ P, int S,
                                                                  long long pstride, int ldp,
                                                                  const bf16_raw* __restrict__ w, float eps,
                                                                  bf16_raw* __restrict__ out, int ldo) {
  constexpr int H = 2048 * NC;
  __shared__ float s_part[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  bf16_raw* hr = h + (size_t)row * ldh;
  const float* pr = P + (size_t)row * ldp;
  u32x4_t hv[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) hv[j] = ld16(hr + (tid + j * 256) * 8);
  float acc[NC][8];
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  for (int s = 0; s < S; ++s) {
    const float* ps = pr + (size_t)s * pstride;
    f32x4_t a[NC][2];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      a[j][0] = *reinterpret_cast<const f32x4_t*>(ps + (tid + j * 256) * 8);
      a[j][1] = *reinterpret_cast<const f32x4_t*>(ps + (tid + j * 256) * 8 + 4);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[j][k] += a[j][0][k];
        acc[j][4 + k] += a[j][1][k];
      }
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    float f[8];
    unpack8(hv[j], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] += acc[j][k];
    hv[j] = pack8(f);
    st16(hr + (tid + j * 256) * 8, hv[j]);
    unpack8(hv[j], f);  // the norm sees the rounded residual, as after EPI_RESID
#pragma unroll
    for (int k = 0; k < 8; ++k) ss += f[k] * f[k];
  }
  if (!out) return;
  ss = wave_sum(ss);
  if ((tid & 63) == 0) s_part[tid >> 6] = ss;
  __syncthreads();
  const float rs = rsqrtf((s_part[0] + s_part[1] + s_part[2] + s_part[3]) / (float)H + eps);
  bf16_raw* orow = out + (size_t)row * ldo;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    float f[8], g[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
    unpack8(hv[j], f);
    if (w) unpack8(ld16(w + (tid + j * 256) * 8), g);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = f[k] * rs * g[k];
    st16(orow + (tid + j * 256) * 8, pack8(f));
  }
}

// Row sums of squares per 64-column block (the layout gemm_sk's fused norm reads, see
// EpiArgs::ss_in): the stage input / embedding of a >128-row forward, whose producer is not a
// residual GEMM. One 64-lane group per row, each lane one block (8 x 16-B loads).
__global__ __launch_bounds__(256) void row_ss_kernel(const bf16_raw* __restrict__ h, int ldh, int rows, int nb,
                                                     float* __restrict__ ss) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), b = threadIdx.x & 63;
  if (row >= rows) return;
  for (int blk = b; blk < nb; blk += 64) {
    const bf16_raw* p = h + (size_t)row * ldh + blk * 64;
    float s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // 16-column units, summed as gemm_sk's residual epilogue does
      float x0[8], x1[8];
      unpack8(ld16(p + j * 16), x0);
      unpack8(ld16(p + j * 16 + 8), x1);
      s4[j] = ss16(x0, x1);
    }
    ss[(size_t)row * nb + blk] = __fadd_rn(__fadd_rn(s4[0], s4[1]), __fadd_rn(s4[2], s4[3]));
  }
}

// Two-pass (mean, then centred variance) over the row held in L2; the optional position add
// rounds to bf16 first, as HF's ``inputs_embeds + position_embeds`` in the model dtype does.
__global__ __launch_bounds__(256) void layernorm_kernel(bf16_raw* __restrict__ x, int ldx,
                                                        const bf16_raw* __restrict__ pe,
                                                        const int* __restrict__ pos,
                                                        const bf16_raw* __restrict__ g,
                                                        const bf16_raw* __restrict__ b, int H,
                                                        float eps, bf16_raw* __restrict__ out,
                                                        int ldo) {
  __shared__ float s_part[2][4];
  const int row = blockIdx.x, tid = threadIdx.x;
  bf16_raw* xr = x + (size_t)row * ldx;
  const bf16_raw* pr = pe ? pe + (size_t)pos[row] * H : nullptr;
  float s = 0.f;
  for (int c = tid; c < (H >> 3); c += 256) {
    float f[8];
    unpack8(ld16(xr + c * 8), f);
    if (pr) {
      float q[8];
      unpack8(ld16(pr + c * 8), q);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += q[j];
      const u32x4_t v = pack8(f);
      st16(xr + c * 8, v);
      unpack8(v, f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[j];
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) s_part[0][tid >> 6] = s;
  __syncthreads();
  const float mu = (s_part[0][0] + s_part[0][1] + s_part[0][2] + s_part[0][3]) / (float)H;
  float v2 = 0.f;
  for (int c = tid; c < (H >> 3); c += 256) {
    float f[8];
    unpack8(ld16(xr + c * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) v2 += (f[j] - mu) * (f[j] - mu);
  }
  v2 = wave_sum(v2);
  if ((tid & 63) == 0) s_part[1][tid >> 6] = v2;
  __syncthreads();
  const float rs = rsqrtf((s_part[1][0] + s_part[1][1] + s_part[1][2] + s_part[1][3]) / (float)H + eps);
  bf16_raw* orow = out + (size_t)row * ldo;
  for (int c = tid; c < (H >> 3); c += 256) {
    float f[8], gg[8], bb[8];
    unpack8(ld16(xr + c * 8), f);
    unpack8(ld16(g + c * 8), gg);
    unpack8(ld16(b + c * 8), bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (f[j] - mu) * rs * gg[j] + bb[j];
    st16(orow + c * 8, pack8(f));
  }
}

// One workgroup; rows <= 1024.
__global__ void argmax_finalize_kernel(unsigned long long* __restrict__ keys, int rows,
                                       int* __restrict__ tokens, int* __restrict__ pos,
                                       int pos_inc, int* __restrict__ history, int hist_stride,
                                       int hist_len, int* __restrict__ step_ctr) {
  const int r = threadIdx.x;
  int step = 0;
  if (step_ctr) step = *step_ctr;
  __syncthreads();
  if (r < rows) {
    const unsigned long long k = keys[r];
    const int tok = (int)argmax_key_index(k);
    keys[r] = 0ull;
    tokens[r] = tok;
    if (pos) pos[r] += pos_inc;
    if (history && step < hist_len) history[(size_t)step * hist_stride + r] = tok;
  }
  if (r == 0 && step_ctr) *step_ctr = step + 1;
}

}  // namespace

extern "C" int lsa_embed(const int* ids, int rows, const void* table, int H, void* out, int ldo,
                         hipStream_t stream) {
  if (rows < 1 || H % 8) return LSA_BAD_SHAPE;
  embed_kernel<<<rows, 256, 0, stream>>>(ids, static_cast<const bf16_raw*>(table), H,
                                        static_cast<bf16_raw*>(out), ldo);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_rmsnorm(const void* x, int ldx, const void* w, int rows, int H, float eps,
                           void* out, int ldo, hipStream_t stream) {
  if (rows < 1 || H % 8) return LSA_BAD_SHAPE;
  const bf16_raw* xb = static_cast<const bf16_raw*>(x);
  const bf16_raw* wb = static_cast<const bf16_raw*>(w);
  bf16_raw* ob = static_cast<bf16_raw*>(out);
  // 16-B row alignment of x/out is what ld16/st16 already assume (ldx, ldo multiples of 8)
  switch (H) {
    case 2048: rmsnorm_reg_kernel<1><<<rows, 256, 0, stream>>>(xb, ldx, wb, eps, ob, ldo); break;
    case 4096: rmsnorm_reg_kernel<2><<<rows, 256, 0, stream>>>(xb, ldx, wb, eps, ob, ldo); break;
    case 6144: rmsnorm_reg_kernel<3><<<rows, 256, 0, stream>>>(xb, ldx, wb, eps, ob, ldo); break;
    case 8192: rmsnorm_reg_kernel<4><<<rows, 256, 0, stream>>>(xb, ldx, wb, eps, ob, ldo); break;
    default:
      rmsnorm_kernel<<<rows, 256, 0, stream>>>(xb, ldx, wb, H, eps, ob, ldo);
  }
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_resid_rmsnorm_partials(void* h, int ldh, const float* partials, int S, long long pstride,
                                          int ldp, const void* w, int rows, int H, float eps, void* out, int ldo,
                                          hipStream_t stream) {
  if (rows < 1 || S < 1 || ldh % 8 || ldp % 8 || (out && ldo % 8) || pstride < (long long)rows * ldp)
    return LSA_BAD_SHAPE;
  bf16_raw* hb = static_cast<bf16_raw*>(h);
  const bf16_raw* wb = static_cast<const bf16_raw*>(w);
  bf16_raw* ob = static_cast<bf16_raw*>(out);
  switch (H) {
    case 2048: resid_norm_partials_kernel<1><<<rows, 256, 0, stream>>>(hb, ldh, partials, S, pstride, ldp, wb, eps, ob, ldo); break;
    case 4096: resid_norm_partials_kernel<2><<<rows, 256, 0, stream>>>(hb, ldh, partials, S, pstride, ldp, wb, eps, ob, ldo); break;
    case 6144: resid_norm_partials_kernel<3><<<rows, 256, 0, stream>>>(hb, ldh, partials, S, pstride, ldp, wb, eps, ob, ldo); break;
    case 8192: resid_norm_partials_kernel<4><<<rows, 256, 0, stream>>>(hb, ldh, partials, S, pstride, ldp, wb, eps, ob, ldo); break;
    default: return LSA_UNSUPPORTED;
  }
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_row_ss(const void* h, int ldh, int rows, int H, float* ss, hipStream_t stream) {
  if (rows < 1 || H % 64 || ldh % 8) return LSA_BAD_SHAPE;
  row_ss_kernel<<<(rows + 3) / 4, 256, 0, stream>>>(static_cast<const bf16_raw*>(h), ldh, rows, H / 64, ss);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_layernorm(void* x, int ldx, const void* pe, const int* pos, const void* g,
                             const void* b, int rows, int H, float eps, void* out, int ldo,
                             hipStream_t stream) {
  if (rows < 1 || H % 8 || !g || !b || (pe && !pos)) return LSA_BAD_SHAPE;
  layernorm_kernel<<<rows, 256, 0, stream>>>(static_cast<bf16_raw*>(x), ldx,
                                            static_cast<const bf16_raw*>(pe), pos,
                                            static_cast<const bf16_raw*>(g),
                                            static_cast<const bf16_raw*>(b), H, eps,
                                            static_cast<bf16_raw*>(out), ldo);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_argmax_finalize(unsigned long long* keys, int rows, int* tokens, int* pos,
                                   int pos_inc, int* history, int hist_stride, int hist_len,
                                   int* step_ctr, hipStream_t stream) {
  if (rows < 1 || rows > 1024) return LSA_BAD_SHAPE;
  const int thr = ((rows + 63) / 64) * 64;
  argmax_finalize_kernel<<<1, thr, 0, stream>>>(keys, rows, tokens, pos, pos_inc, history,
                                               hist_stride, hist_len, step_ctr);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

namespace {
__global__ void pos_advance_kernel(int* __restrict__ pos, int rows, int inc) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) pos[r] += inc;
}
}  // namespace

// Device-side position counters of a pipeline stage (its KV length per row) - advanced inside
// the captured decode graph, so replays never need host-side re-capture.
extern "C" int lsa_pos_advance(int* pos, int rows, int inc, hipStream_t stream) {
  if (rows < 1) return LSA_BAD_SHAPE;
  pos_advance_kernel<<<(rows + 255) / 256, 256, 0, stream>>>(pos, rows, inc);
  LSA_CHECK_LAUNCH();
  return LSA_OK;
}

extern "C" int lsa_version() { return 1; }
