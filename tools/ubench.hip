// Instruction-rate microbenchmarks on gfx950 (design study for the Fp
// product; not part of the library).  Each kernel runs `iters` rounds of 8
// independent chains per lane; prints lane-ops/s per instruction form.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip && ./tools/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHAINS 8

__global__ void __launch_bounds__(256) k_mad64(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a[CHAINS];
  for (int k = 0; k < CHAINS; k++) a[k] = io[i] + k;
  const uint32_t m = (uint32_t)a[0] | 1u;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) a[k] = (uint64_t)(uint32_t)a[k] * m + (a[k] >> 32);
  uint64_t x = 0;
  for (int k = 0; k < CHAINS; k++) x ^= a[k];
  io[i] = x;
}

// mad64 chains with 2 independent full-rate adds per mad (the product's overhead mix)
__global__ void __launch_bounds__(256) k_mad64_mix(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a[CHAINS];
  uint32_t s[CHAINS];
  for (int k = 0; k < CHAINS; k++) { a[k] = io[i] + k; s[k] = (uint32_t)io[i] ^ k; }
  const uint32_t m = (uint32_t)a[0] | 1u;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) {
      a[k] = (uint64_t)(uint32_t)a[k] * m + (a[k] >> 32);
      s[k] = (s[k] ^ (uint32_t)t) + 0x9e3779b9u;
    }
  uint64_t x = 0;
  for (int k = 0; k < CHAINS; k++) x ^= a[k] ^ s[k];
  io[i] = x;
}

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_dot2(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc[CHAINS];
  us2 x, y;
  x.x = (unsigned short)io[i]; x.y = (unsigned short)(io[i] >> 16);
  y.x = (unsigned short)(io[i] >> 32); y.y = (unsigned short)(io[i] >> 48);
  for (int k = 0; k < CHAINS; k++) acc[k] = (uint32_t)io[i] + k;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) acc[k] = __builtin_amdgcn_udot2(x, y, acc[k] >> 1, false);
  uint32_t r = 0;
  for (int k = 0; k < CHAINS; k++) r ^= acc[k];
  io[i] = r;
}

__global__ void __launch_bounds__(256) k_mul24(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[CHAINS];
  for (int k = 0; k < CHAINS; k++) a[k] = (uint32_t)io[i] + k;
  const uint32_t m = ((uint32_t)io[i] | 1u) & 0xffffffu;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) a[k] = __umul24(a[k], m) + (a[k] >> 9);
  uint32_t r = 0;
  for (int k = 0; k < CHAINS; k++) r ^= a[k];
  io[i] = r;
}

__global__ void __launch_bounds__(256) k_mulhi24(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[CHAINS];
  for (int k = 0; k < CHAINS; k++) a[k] = (uint32_t)io[i] + k;
  const uint32_t m = ((uint32_t)io[i] | 1u) & 0xffffffu;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) a[k] = __umulhi(a[k] & 0xffffffu, m) ^ a[k];
  uint32_t r = 0;
  for (int k = 0; k < CHAINS; k++) r ^= a[k];
  io[i] = r;
}

__global__ void __launch_bounds__(256) k_add32(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[CHAINS];
  for (int k = 0; k < CHAINS; k++) a[k] = (uint32_t)io[i] + k;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) a[k] = (a[k] ^ t) + 0x9e3779b9u;
  uint32_t r = 0;
  for (int k = 0; k < CHAINS; k++) r ^= a[k];
  io[i] = r;
}

__global__ void __launch_bounds__(256) k_fma64(uint64_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  double a[CHAINS];
  for (int k = 0; k < CHAINS; k++) a[k] = (double)(io[i] + k);
  const double m = 1.0000001, c = 0.5;
  for (uint32_t t = 0; t < iters; t++)
#pragma unroll
    for (int k = 0; k < CHAINS; k++) a[k] = __builtin_fma(a[k], m, c);
  double r = 0;
  for (int k = 0; k < CHAINS; k++) r += a[k];
  io[i] = (uint64_t)r;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static double run(kfn k, uint64_t* buf, uint32_t lanes, uint32_t iters, int ops_per_chain_iter) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(lanes / 256), dim3(256), 0, 0, buf, 16u);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(k, dim3(lanes / 256), dim3(256), 0, 0, buf, iters);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return (double)lanes * iters * CHAINS * ops_per_chain_iter / (ms * 1e-3);
}

int main() {
  const uint32_t lanes = 256 * 256 * 8, iters = 4096;
  uint64_t* buf;
  if (hipMalloc((void**)&buf, (size_t)lanes * 8) != hipSuccess) return 1;
  hipMemset(buf, 0x5a, (size_t)lanes * 8);
  printf("{\"lanes\": %u, \"iters\": %u, \"chains\": %d,\n", lanes, iters, CHAINS);
  printf(" \"mad_u64_u32\": %.4g,\n", run(k_mad64, buf, lanes, iters, 1));
  printf(" \"mad_u64_u32_with_2_adds_mads_per_s\": %.4g,\n", run(k_mad64_mix, buf, lanes, iters, 1));
  printf(" \"dot2_u32_u16\": %.4g,\n", run(k_dot2, buf, lanes, iters, 1));
  printf(" \"mul_u32_u24\": %.4g,\n", run(k_mul24, buf, lanes, iters, 1));
  printf(" \"mulhi_u32_u24\": %.4g,\n", run(k_mulhi24, buf, lanes, iters, 1));
  printf(" \"add_u32_pairs\": %.4g,\n", run(k_add32, buf, lanes, iters, 1));
  printf(" \"fma_f64\": %.4g}\n", run(k_fma64, buf, lanes, iters, 1));
  hipFree(buf);
  return 0;
}
