#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>

#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50"
__global__ void case_0(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_1(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_2(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_3(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_4(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_5(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_6(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_7(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_8(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_9(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_10(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_11(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_12(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_13(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_14(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_15(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_16(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_17(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_18(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_19(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_20(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_21(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_22(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_23(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_24(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_25(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_26(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_27(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_28(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_29(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_30(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_31(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_32(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_33(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_34(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v40, v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_35(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_36(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_37(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_38(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_39(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_40(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_41(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_42(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_43(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_44(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_45(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_46(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_47(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_48(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_49(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_50(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_51(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_52(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_53(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_54(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_55(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_56(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_57(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_58(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_59(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_60(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_61(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_62(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_63(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_64(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_65(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_66(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_67(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_68(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_69(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_add_f32 v41, v41, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_70(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_71(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_72(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_73(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_74(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_75(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_76(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_77(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_78(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_79(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_80(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_81(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_82(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_83(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_84(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_85(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_86(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_87(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_88(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_89(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_90(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_91(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_92(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_93(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_94(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_95(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_96(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_97(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_98(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_99(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_100(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_101(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_102(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_103(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_104(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_fma_f32 v40, v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_105(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_106(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_107(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_108(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_109(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_110(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_111(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_112(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_113(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_114(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_115(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_116(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_117(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_118(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_119(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_120(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_121(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_122(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_123(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_124(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_125(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_126(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_127(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_128(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_129(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_130(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_131(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_132(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_133(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_134(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_135(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_136(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_137(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_138(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_139(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v40, %[e] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_140(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_141(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_142(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_143(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_144(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_145(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_146(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_147(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_148(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_149(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_150(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_151(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_152(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_153(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_154(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_155(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_156(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_157(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_158(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_159(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_160(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_161(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_162(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_163(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_164(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_165(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_166(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_167(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_168(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_169(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_170(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_171(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_172(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_173(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_174(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_exp_f32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_175(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_176(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_177(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_178(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_179(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_180(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_181(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_182(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_183(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_184(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_185(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_186(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_187(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_188(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_189(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_190(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_191(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_192(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_193(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_194(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_195(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_196(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_197(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_198(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_199(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_200(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_201(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_202(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_203(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_204(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_205(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_206(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_207(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_208(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_209(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_cvt_pk_bf16_f32 v40, %[e], %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_210(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_211(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_212(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_213(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_214(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_215(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_216(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_217(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_218(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_219(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_220(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_221(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_222(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_223(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_224(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_225(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_226(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_227(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_228(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_229(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_230(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_231(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_232(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_233(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_234(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_235(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_236(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_237(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_238(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_239(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_240(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_241(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_242(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_243(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_244(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_245(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_246(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_247(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_248(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_249(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_250(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_251(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n \n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_252(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_253(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_254(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_255(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_256(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_257(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_258(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 0\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_259(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_260(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_261(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_262(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_263(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_264(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_265(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_266(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_267(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_268(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_269(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_270(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_271(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_272(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 1\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_273(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_add_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_274(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_275(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[40:41], v[42:43], v[46:47]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_276(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_fma_f32 v[44:45], v[42:43], v[46:47], v[40:41]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_277(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_pk_mov_b32 v[44:45], v[40:41], v[42:43] op_sel:[0,1]\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_278(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_add_f32 v44, v40, v42\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
__global__ void case_279(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned nb = 0;
  for (int it = 0; it < iters; ++it) {
    const float a = in[(i * 5 + it * 7) & 4095], b = in[(i * 3 + it * 11 + 1) & 4095], c = in[(i + it * 13 + 2) & 4095],
                d = in[(i * 7 + it * 17 + 3) & 4095], e = in[(i * 11 + it * 19 + 4) & 4095];
    float h0, h1, s0, s1;
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n v_mov_b32 v48, v49\n v_mov_b32 v50, v49\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(h0), [o1] "=v"(h1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    asm volatile("v_mov_b32 v40, %[a]\n v_mov_b32 v41, %[b]\n v_mov_b32 v42, %[c]\n v_mov_b32 v43, %[d]\n v_mov_b32 v46, %[d]\n v_mov_b32 v47, %[c]\n v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v49, %[a]\n s_nop 7\n s_nop 7\n v_mov_b32 v40, %[e]\n s_nop 7\n s_nop 7\n v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_nop 7\n v_mov_b32 %[o0], v44\n v_mov_b32 %[o1], v45\n" : [o0] "=v"(s0), [o1] "=v"(s1) : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e) : CLOB);
    unsigned x0, x1, y0, y1;
    memcpy(&x0, &h0, 4); memcpy(&x1, &h1, 4); memcpy(&y0, &s0, 4); memcpy(&y1, &s1, 4);
    nb += (x0 != y0) + (x1 != y1);
  }
  bad[i] = nb;
}
typedef void (*KFn)(const float*, unsigned*, int);
static const KFn KS[] = {case_0, case_1, case_2, case_3, case_4, case_5, case_6, case_7, case_8, case_9, case_10, case_11, case_12, case_13, case_14, case_15, case_16, case_17, case_18, case_19, case_20, case_21, case_22, case_23, case_24, case_25, case_26, case_27, case_28, case_29, case_30, case_31, case_32, case_33, case_34, case_35, case_36, case_37, case_38, case_39, case_40, case_41, case_42, case_43, case_44, case_45, case_46, case_47, case_48, case_49, case_50, case_51, case_52, case_53, case_54, case_55, case_56, case_57, case_58, case_59, case_60, case_61, case_62, case_63, case_64, case_65, case_66, case_67, case_68, case_69, case_70, case_71, case_72, case_73, case_74, case_75, case_76, case_77, case_78, case_79, case_80, case_81, case_82, case_83, case_84, case_85, case_86, case_87, case_88, case_89, case_90, case_91, case_92, case_93, case_94, case_95, case_96, case_97, case_98, case_99, case_100, case_101, case_102, case_103, case_104, case_105, case_106, case_107, case_108, case_109, case_110, case_111, case_112, case_113, case_114, case_115, case_116, case_117, case_118, case_119, case_120, case_121, case_122, case_123, case_124, case_125, case_126, case_127, case_128, case_129, case_130, case_131, case_132, case_133, case_134, case_135, case_136, case_137, case_138, case_139, case_140, case_141, case_142, case_143, case_144, case_145, case_146, case_147, case_148, case_149, case_150, case_151, case_152, case_153, case_154, case_155, case_156, case_157, case_158, case_159, case_160, case_161, case_162, case_163, case_164, case_165, case_166, case_167, case_168, case_169, case_170, case_171, case_172, case_173, case_174, case_175, case_176, case_177, case_178, case_179, case_180, case_181, case_182, case_183, case_184, case_185, case_186, case_187, case_188, case_189, case_190, case_191, case_192, case_193, case_194, case_195, case_196, case_197, case_198, case_199, case_200, case_201, case_202, case_203, case_204, case_205, case_206, case_207, case_208, case_209, case_210, case_211, case_212, case_213, case_214, case_215, case_216, case_217, case_218, case_219, case_220, case_221, case_222, case_223, case_224, case_225, case_226, case_227, case_228, case_229, case_230, case_231, case_232, case_233, case_234, case_235, case_236, case_237, case_238, case_239, case_240, case_241, case_242, case_243, case_244, case_245, case_246, case_247, case_248, case_249, case_250, case_251, case_252, case_253, case_254, case_255, case_256, case_257, case_258, case_259, case_260, case_261, case_262, case_263, case_264, case_265, case_266, case_267, case_268, case_269, case_270, case_271, case_272, case_273, case_274, case_275, case_276, case_277, case_278, case_279};
static const char* NAMES[] = {"valu32_lo 0 pk_add", "valu32_lo 0 pk_mul", "valu32_lo 0 pk_fma_src0", "valu32_lo 0 pk_fma_src2", "valu32_lo 0 pk_mov", "valu32_lo 0 add_f32", "valu32_lo 0 dpp_read", "valu32_lo nop0 pk_add", "valu32_lo nop0 pk_mul", "valu32_lo nop0 pk_fma_src0", "valu32_lo nop0 pk_fma_src2", "valu32_lo nop0 pk_mov", "valu32_lo nop0 add_f32", "valu32_lo nop0 dpp_read", "valu32_lo valu1 pk_add", "valu32_lo valu1 pk_mul", "valu32_lo valu1 pk_fma_src0", "valu32_lo valu1 pk_fma_src2", "valu32_lo valu1 pk_mov", "valu32_lo valu1 add_f32", "valu32_lo valu1 dpp_read", "valu32_lo nop1 pk_add", "valu32_lo nop1 pk_mul", "valu32_lo nop1 pk_fma_src0", "valu32_lo nop1 pk_fma_src2", "valu32_lo nop1 pk_mov", "valu32_lo nop1 add_f32", "valu32_lo nop1 dpp_read", "valu32_lo valu2 pk_add", "valu32_lo valu2 pk_mul", "valu32_lo valu2 pk_fma_src0", "valu32_lo valu2 pk_fma_src2", "valu32_lo valu2 pk_mov", "valu32_lo valu2 add_f32", "valu32_lo valu2 dpp_read", "valu32_hi 0 pk_add", "valu32_hi 0 pk_mul", "valu32_hi 0 pk_fma_src0", "valu32_hi 0 pk_fma_src2", "valu32_hi 0 pk_mov", "valu32_hi 0 add_f32", "valu32_hi 0 dpp_read", "valu32_hi nop0 pk_add", "valu32_hi nop0 pk_mul", "valu32_hi nop0 pk_fma_src0", "valu32_hi nop0 pk_fma_src2", "valu32_hi nop0 pk_mov", "valu32_hi nop0 add_f32", "valu32_hi nop0 dpp_read", "valu32_hi valu1 pk_add", "valu32_hi valu1 pk_mul", "valu32_hi valu1 pk_fma_src0", "valu32_hi valu1 pk_fma_src2", "valu32_hi valu1 pk_mov", "valu32_hi valu1 add_f32", "valu32_hi valu1 dpp_read", "valu32_hi nop1 pk_add", "valu32_hi nop1 pk_mul", "valu32_hi nop1 pk_fma_src0", "valu32_hi nop1 pk_fma_src2", "valu32_hi nop1 pk_mov", "valu32_hi nop1 add_f32", "valu32_hi nop1 dpp_read", "valu32_hi valu2 pk_add", "valu32_hi valu2 pk_mul", "valu32_hi valu2 pk_fma_src0", "valu32_hi valu2 pk_fma_src2", "valu32_hi valu2 pk_mov", "valu32_hi valu2 add_f32", "valu32_hi valu2 dpp_read", "vop3_fma_lo 0 pk_add", "vop3_fma_lo 0 pk_mul", "vop3_fma_lo 0 pk_fma_src0", "vop3_fma_lo 0 pk_fma_src2", "vop3_fma_lo 0 pk_mov", "vop3_fma_lo 0 add_f32", "vop3_fma_lo 0 dpp_read", "vop3_fma_lo nop0 pk_add", "vop3_fma_lo nop0 pk_mul", "vop3_fma_lo nop0 pk_fma_src0", "vop3_fma_lo nop0 pk_fma_src2", "vop3_fma_lo nop0 pk_mov", "vop3_fma_lo nop0 add_f32", "vop3_fma_lo nop0 dpp_read", "vop3_fma_lo valu1 pk_add", "vop3_fma_lo valu1 pk_mul", "vop3_fma_lo valu1 pk_fma_src0", "vop3_fma_lo valu1 pk_fma_src2", "vop3_fma_lo valu1 pk_mov", "vop3_fma_lo valu1 add_f32", "vop3_fma_lo valu1 dpp_read", "vop3_fma_lo nop1 pk_add", "vop3_fma_lo nop1 pk_mul", "vop3_fma_lo nop1 pk_fma_src0", "vop3_fma_lo nop1 pk_fma_src2", "vop3_fma_lo nop1 pk_mov", "vop3_fma_lo nop1 add_f32", "vop3_fma_lo nop1 dpp_read", "vop3_fma_lo valu2 pk_add", "vop3_fma_lo valu2 pk_mul", "vop3_fma_lo valu2 pk_fma_src0", "vop3_fma_lo valu2 pk_fma_src2", "vop3_fma_lo valu2 pk_mov", "vop3_fma_lo valu2 add_f32", "vop3_fma_lo valu2 dpp_read", "dpp_lo 0 pk_add", "dpp_lo 0 pk_mul", "dpp_lo 0 pk_fma_src0", "dpp_lo 0 pk_fma_src2", "dpp_lo 0 pk_mov", "dpp_lo 0 add_f32", "dpp_lo 0 dpp_read", "dpp_lo nop0 pk_add", "dpp_lo nop0 pk_mul", "dpp_lo nop0 pk_fma_src0", "dpp_lo nop0 pk_fma_src2", "dpp_lo nop0 pk_mov", "dpp_lo nop0 add_f32", "dpp_lo nop0 dpp_read", "dpp_lo valu1 pk_add", "dpp_lo valu1 pk_mul", "dpp_lo valu1 pk_fma_src0", "dpp_lo valu1 pk_fma_src2", "dpp_lo valu1 pk_mov", "dpp_lo valu1 add_f32", "dpp_lo valu1 dpp_read", "dpp_lo nop1 pk_add", "dpp_lo nop1 pk_mul", "dpp_lo nop1 pk_fma_src0", "dpp_lo nop1 pk_fma_src2", "dpp_lo nop1 pk_mov", "dpp_lo nop1 add_f32", "dpp_lo nop1 dpp_read", "dpp_lo valu2 pk_add", "dpp_lo valu2 pk_mul", "dpp_lo valu2 pk_fma_src0", "dpp_lo valu2 pk_fma_src2", "dpp_lo valu2 pk_mov", "dpp_lo valu2 add_f32", "dpp_lo valu2 dpp_read", "trans_lo 0 pk_add", "trans_lo 0 pk_mul", "trans_lo 0 pk_fma_src0", "trans_lo 0 pk_fma_src2", "trans_lo 0 pk_mov", "trans_lo 0 add_f32", "trans_lo 0 dpp_read", "trans_lo nop0 pk_add", "trans_lo nop0 pk_mul", "trans_lo nop0 pk_fma_src0", "trans_lo nop0 pk_fma_src2", "trans_lo nop0 pk_mov", "trans_lo nop0 add_f32", "trans_lo nop0 dpp_read", "trans_lo valu1 pk_add", "trans_lo valu1 pk_mul", "trans_lo valu1 pk_fma_src0", "trans_lo valu1 pk_fma_src2", "trans_lo valu1 pk_mov", "trans_lo valu1 add_f32", "trans_lo valu1 dpp_read", "trans_lo nop1 pk_add", "trans_lo nop1 pk_mul", "trans_lo nop1 pk_fma_src0", "trans_lo nop1 pk_fma_src2", "trans_lo nop1 pk_mov", "trans_lo nop1 add_f32", "trans_lo nop1 dpp_read", "trans_lo valu2 pk_add", "trans_lo valu2 pk_mul", "trans_lo valu2 pk_fma_src0", "trans_lo valu2 pk_fma_src2", "trans_lo valu2 pk_mov", "trans_lo valu2 add_f32", "trans_lo valu2 dpp_read", "cvt_pk_lo 0 pk_add", "cvt_pk_lo 0 pk_mul", "cvt_pk_lo 0 pk_fma_src0", "cvt_pk_lo 0 pk_fma_src2", "cvt_pk_lo 0 pk_mov", "cvt_pk_lo 0 add_f32", "cvt_pk_lo 0 dpp_read", "cvt_pk_lo nop0 pk_add", "cvt_pk_lo nop0 pk_mul", "cvt_pk_lo nop0 pk_fma_src0", "cvt_pk_lo nop0 pk_fma_src2", "cvt_pk_lo nop0 pk_mov", "cvt_pk_lo nop0 add_f32", "cvt_pk_lo nop0 dpp_read", "cvt_pk_lo valu1 pk_add", "cvt_pk_lo valu1 pk_mul", "cvt_pk_lo valu1 pk_fma_src0", "cvt_pk_lo valu1 pk_fma_src2", "cvt_pk_lo valu1 pk_mov", "cvt_pk_lo valu1 add_f32", "cvt_pk_lo valu1 dpp_read", "cvt_pk_lo nop1 pk_add", "cvt_pk_lo nop1 pk_mul", "cvt_pk_lo nop1 pk_fma_src0", "cvt_pk_lo nop1 pk_fma_src2", "cvt_pk_lo nop1 pk_mov", "cvt_pk_lo nop1 add_f32", "cvt_pk_lo nop1 dpp_read", "cvt_pk_lo valu2 pk_add", "cvt_pk_lo valu2 pk_mul", "cvt_pk_lo valu2 pk_fma_src0", "cvt_pk_lo valu2 pk_fma_src2", "cvt_pk_lo valu2 pk_mov", "cvt_pk_lo valu2 add_f32", "cvt_pk_lo valu2 dpp_read", "pk_add 0 pk_add", "pk_add 0 pk_mul", "pk_add 0 pk_fma_src0", "pk_add 0 pk_fma_src2", "pk_add 0 pk_mov", "pk_add 0 add_f32", "pk_add 0 dpp_read", "pk_add nop0 pk_add", "pk_add nop0 pk_mul", "pk_add nop0 pk_fma_src0", "pk_add nop0 pk_fma_src2", "pk_add nop0 pk_mov", "pk_add nop0 add_f32", "pk_add nop0 dpp_read", "pk_add valu1 pk_add", "pk_add valu1 pk_mul", "pk_add valu1 pk_fma_src0", "pk_add valu1 pk_fma_src2", "pk_add valu1 pk_mov", "pk_add valu1 add_f32", "pk_add valu1 dpp_read", "pk_add nop1 pk_add", "pk_add nop1 pk_mul", "pk_add nop1 pk_fma_src0", "pk_add nop1 pk_fma_src2", "pk_add nop1 pk_mov", "pk_add nop1 add_f32", "pk_add nop1 dpp_read", "pk_add valu2 pk_add", "pk_add valu2 pk_mul", "pk_add valu2 pk_fma_src0", "pk_add valu2 pk_fma_src2", "pk_add valu2 pk_mov", "pk_add valu2 add_f32", "pk_add valu2 dpp_read", "mov_lo 0 pk_add", "mov_lo 0 pk_mul", "mov_lo 0 pk_fma_src0", "mov_lo 0 pk_fma_src2", "mov_lo 0 pk_mov", "mov_lo 0 add_f32", "mov_lo 0 dpp_read", "mov_lo nop0 pk_add", "mov_lo nop0 pk_mul", "mov_lo nop0 pk_fma_src0", "mov_lo nop0 pk_fma_src2", "mov_lo nop0 pk_mov", "mov_lo nop0 add_f32", "mov_lo nop0 dpp_read", "mov_lo valu1 pk_add", "mov_lo valu1 pk_mul", "mov_lo valu1 pk_fma_src0", "mov_lo valu1 pk_fma_src2", "mov_lo valu1 pk_mov", "mov_lo valu1 add_f32", "mov_lo valu1 dpp_read", "mov_lo nop1 pk_add", "mov_lo nop1 pk_mul", "mov_lo nop1 pk_fma_src0", "mov_lo nop1 pk_fma_src2", "mov_lo nop1 pk_mov", "mov_lo nop1 add_f32", "mov_lo nop1 dpp_read", "mov_lo valu2 pk_add", "mov_lo valu2 pk_mul", "mov_lo valu2 pk_fma_src0", "mov_lo valu2 pk_fma_src2", "mov_lo valu2 pk_mov", "mov_lo valu2 add_f32", "mov_lo valu2 dpp_read"};
int main() {
  const int N = 4096, ITERS = 64;
  std::vector<float> h(N);
  unsigned s = 12345u;
  for (int i = 0; i < N; ++i) { s = s * 1664525u + 1013904223u; h[i] = ((s >> 8) & 0xffff) / 4096.0f - 8.0f + 0.001f * i; }
  float* din; unsigned* dbad;
  hipMalloc(&din, N * 4);
  const int MAXT = 256 * 8 * 256;
  hipMalloc(&dbad, MAXT * 4);
  hipMemcpy(din, h.data(), N * 4, hipMemcpyHostToDevice);
  std::vector<unsigned> hb(MAXT);
  // (blocks, threads): one wave per SIMD (1024 x 64) and 8 waves per SIMD (1024 x 512)
  const int cfg[2][2] = {{1024, 64}, {1024, 512}};
  for (int c = 0; c < 280; ++c) {
    unsigned long long tot[2] = {0, 0}, tested[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
      const int nb = cfg[k][0], nt = cfg[k][1];
      hipLaunchKernelGGL(KS[c], dim3(nb), dim3(nt), 0, 0, din, dbad, ITERS);
      if (hipDeviceSynchronize() != hipSuccess) { printf("case %d failed\n", c); return 2; }
      hipMemcpy(hb.data(), dbad, (size_t)nb * nt * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < nb * nt; ++i) tot[k] += hb[i];
      tested[k] = 2ull * nb * nt * ITERS;
    }
    printf("%-40s 1w/SIMD %llu/%llu  8w/SIMD %llu/%llu\n", NAMES[c], tot[0], tested[0], tot[1], tested[1]);
  }
  hipFree(din); hipFree(dbad);
  return 0;
}
