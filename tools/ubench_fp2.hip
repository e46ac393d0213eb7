// Design study (not part of the library): the Fp2 product as Karatsuba over
// the library's Fp leaf (3 calls, 2 lazy additions, 3 modular subtractions)
// against ONE Fp2 leaf computing each output coefficient as a sum of two
// products with a single Montgomery reduction (fp2.h fp2_mul_sop):
//   c0 = a0 b0 + (2p - a1) b1,  c1 = a0 b1 + a1 b0    (4 x 196 + 2 x 196 digit mads)
// (A Karatsuba on double-width columns with one reduction per coefficient,
// 980 digit mads, measured 4.40 us lone / 9.9 G/s: its signed 28-column
// accumulators spill; not kept, profiles/r06j_ubench_fp2.json.)
// The Fp2 leaf's 48 argument dwords exceed the 32 argument VGPRs of the
// AMDGPU calling convention, so 16 travel on the stack (variant "stack"); the
// "ptr" variant passes b by pointer.  Lone-wave latency and full-chip
// throughput of chains of Fp2 products.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_fp2 tools/ubench_fp2.hip && ./tools/ubench_fp2
#define BGV_FPMUL_CALL 1
#define BGV_FP2_LEAF 0  // fp2_mul_inl stays Karatsuba over the Fp leaf (the baseline)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../lodestar_amd/csrc/fp2.h"

namespace bgv {

typedef uint32_t fp2_vec_t __attribute__((ext_vector_type(24)));

static __device__ __noinline__ fp2_vec_t fp2_mul_leaf_stack(fp_vec_t a0, fp_vec_t a1, fp_vec_t b0, fp_vec_t b1) {
  fp2_t a, b, r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    a.c0.l[i] = a0[i]; a.c1.l[i] = a1[i]; b.c0.l[i] = b0[i]; b.c1.l[i] = b1[i];
  }
  fp2_mul_sop(r, a, b);
  fp2_vec_t v;
#pragma unroll
  for (int i = 0; i < NL; i++) { v[i] = r.c0.l[i]; v[NL + i] = r.c1.l[i]; }
  return v;
}

static __device__ __noinline__ fp2_vec_t fp2_mul_leaf_ptr(fp_vec_t a0, fp_vec_t a1, const fp2_t* bp) {
  fp2_t a, r;
#pragma unroll
  for (int i = 0; i < NL; i++) { a.c0.l[i] = a0[i]; a.c1.l[i] = a1[i]; }
  const fp2_t b = *bp;
  fp2_mul_sop(r, a, b);
  fp2_vec_t v;
#pragma unroll
  for (int i = 0; i < NL; i++) { v[i] = r.c0.l[i]; v[NL + i] = r.c1.l[i]; }
  return v;
}

}  // namespace bgv

using namespace bgv;

__device__ __forceinline__ void to_vec(fp_vec_t& v, const fp_t& a) {
#pragma unroll
  for (int i = 0; i < NL; i++) v[i] = a.l[i];
}

__global__ void __launch_bounds__(64) k_fp2_kara(fp2_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp2_t x = io[2 * i], y = io[2 * i + 1];
  for (uint32_t t = 0; t < iters; t++) fp2_mul_inl(x, x, y);
  io[2 * i] = x;
}

__global__ void __launch_bounds__(64) k_fp2_stack(fp2_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp2_t x = io[2 * i], y = io[2 * i + 1];
  fp_vec_t y0, y1;
  to_vec(y0, y.c0);
  to_vec(y1, y.c1);
  for (uint32_t t = 0; t < iters; t++) {
    fp_vec_t x0, x1;
    to_vec(x0, x.c0);
    to_vec(x1, x.c1);
    const fp2_vec_t r = fp2_mul_leaf_stack(x0, x1, y0, y1);
#pragma unroll
    for (int k = 0; k < NL; k++) { x.c0.l[k] = r[k]; x.c1.l[k] = r[NL + k]; }
  }
  io[2 * i] = x;
}

__global__ void __launch_bounds__(64) k_fp2_ptr(fp2_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp2_t x = io[2 * i];
  const fp2_t* yp = &io[2 * i + 1];
  for (uint32_t t = 0; t < iters; t++) {
    fp_vec_t x0, x1;
    to_vec(x0, x.c0);
    to_vec(x1, x.c1);
    const fp2_vec_t r = fp2_mul_leaf_ptr(x0, x1, yp);
#pragma unroll
    for (int k = 0; k < NL; k++) { x.c0.l[k] = r[k]; x.c1.l[k] = r[NL + k]; }
  }
  io[2 * i] = x;
}

// correctness: the three forms agree on random canonical operands
__global__ void k_check(const fp2_t* in, uint32_t* bad, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fp2_t x = in[2 * i], y = in[2 * i + 1];
  fp2_t r0;
  fp2_mul_inl(r0, x, y);
  fp_vec_t x0, x1, y0, y1;
  to_vec(x0, x.c0); to_vec(x1, x.c1); to_vec(y0, y.c0); to_vec(y1, y.c1);
  const fp2_vec_t r1 = fp2_mul_leaf_stack(x0, x1, y0, y1);
  const fp2_vec_t r2 = fp2_mul_leaf_ptr(x0, x1, &in[2 * i + 1]);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; k++)
    acc |= (r0.c0.l[k] ^ r1[k]) | (r0.c1.l[k] ^ r1[NL + k]) | (r0.c0.l[k] ^ r2[k]) | (r0.c1.l[k] ^ r2[NL + k]);
  if (acc) atomicAdd(bad, 1u);
}

static float run(void (*k)(fp2_t*, uint32_t), fp2_t* d, uint32_t blocks, uint32_t iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, 8u);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  const uint32_t big = 1024 * 8;  // 8 waves per SIMD
  const size_t n = (size_t)big * 64;
  fp2_t* d;
  hipMalloc(&d, n * 2 * sizeof(fp2_t));
  // canonical random operands (top limb below p's)
  fp2_t* h = (fp2_t*)malloc(n * 2 * sizeof(fp2_t));
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < n * 2; i++) {
    fp_t* c[2] = {&h[i].c0, &h[i].c1};
    for (int q = 0; q < 2; q++)
      for (int k = 0; k < NL; k++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        c[q]->l[k] = (uint32_t)s;
        if (k == NL - 1) c[q]->l[k] &= 0x0fffffffu;
      }
  }
  hipMemcpy(d, h, n * 2 * sizeof(fp2_t), hipMemcpyHostToDevice);
  uint32_t* bad;
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(k_check, dim3((uint32_t)(n / 64)), dim3(64), 0, 0, d, bad, (uint32_t)n);
  uint32_t hb = 0;
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  const uint32_t it = 2000;
  struct { const char* name; float lone, thr; } r[3];
  hipMemcpy(d, h, n * 2 * sizeof(fp2_t), hipMemcpyHostToDevice);
  r[0] = {"karatsuba_3_fp_leaves", run(k_fp2_kara, d, 1, it), run(k_fp2_kara, d, big, it / 10)};
  hipMemcpy(d, h, n * 2 * sizeof(fp2_t), hipMemcpyHostToDevice);
  r[1] = {"fp2_leaf_stack_args", run(k_fp2_stack, d, 1, it), run(k_fp2_stack, d, big, it / 10)};
  hipMemcpy(d, h, n * 2 * sizeof(fp2_t), hipMemcpyHostToDevice);
  r[2] = {"fp2_leaf_b_by_pointer", run(k_fp2_ptr, d, 1, it), run(k_fp2_ptr, d, big, it / 10)};

  printf("{\"mismatches\": %u, ", hb);
  for (int k = 0; k < 3; k++) {
    const double lone_us = r[k].lone * 1e3 / it;
    const double thr = (double)big * 64 * (it / 10) / (r[k].thr * 1e-3) / 1e9;
    printf("%s\"%s\": {\"lone_wave_us_per_fp2_mul\": %.4f, \"chip_G_fp2_mul_per_s\": %.3f}", k ? ", " : "", r[k].name, lone_us, thr);
  }
  printf("}\n");
  return 0;
}
