// Latency microbenchmarks of the cooperative building blocks (design study
// for the latency path; not part of the library):
//   * a lone wave's chain of dependent Fp products (the product latency);
//   * c_mul (fp12_coop.h, 128 lanes) in a loop: the latency of one
//     cooperative Fp12 product, and of its rounds taken apart.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_coop tools/ubench_coop.hip
#define BGV_FPMUL_CALL 0
#include "../lodestar_amd/csrc/bgv_internal.h"
#include "../lodestar_amd/csrc/fp12_coop.h"
#include <stdio.h>

using namespace bgv;

__global__ void __launch_bounds__(64) k_chain(fp_t* io, uint32_t iters) {
  fp_t x = io[threadIdx.x], y = io[64 + threadIdx.x];
  for (uint32_t k = 0; k < iters; k++) fp_mul(x, x, y);
  io[threadIdx.x] = x;
}

__global__ void __launch_bounds__(64) k_chain_add(fp_t* io, uint32_t iters) {
  fp_t x = io[threadIdx.x], y = io[64 + threadIdx.x];
  for (uint32_t k = 0; k < iters; k++) fp_add(x, x, y);
  io[threadIdx.x] = x;
}

// one lane: the Fp12 inversion at the start of the final exponentiation
__global__ void __launch_bounds__(64) k_inv(const fp12_t* in, fp12_t* out, uint32_t iters) {
  fp12_t x = in[0];
  for (uint32_t k = 0; k < iters; k++) fp12_inv(x, x);
  if (threadIdx.x == 0) out[0] = x;
}

// one workgroup: a whole final exponentiation (k_batch_final's body)
__global__ void __launch_bounds__(128) k_fe(const fp12_t* in, fp12_t* out, uint32_t iters) {
  __shared__ cscratch s;
  fp12_t x = in[0];
  for (uint32_t k = 0; k < iters; k++) {
    __shared__ fp12_t r;
    c_final_exp(&r, x, &s);
    x = r;
  }
  if (threadIdx.x == 0) out[0] = x;
}

// mode 0: full c_mul; 1: round 1 only (108 products + barrier)
__global__ void __launch_bounds__(128) k_cmul(const fp12_t* in, fp12_t* out, uint32_t iters, uint32_t mode) {
  __shared__ cscratch s;
  __shared__ wfp12 a, b;
  c_load(&a, in[0]);
  c_load(&b, in[1]);
  for (uint32_t k = 0; k < iters; k++) {
    if (mode == 0) {
      c_mul(&a, &a, &b, &s);
    } else {
      const uint32_t l = threadIdx.x;
      if (l < 108) {
        const uint32_t p = l / 3, i = p / 6;
        fp_t r;
        fp_mul(r, a.c[i].c0, b.c[i].c1);
        s.p[l] = r;
      }
      __syncthreads();
      if (l < 12) a.c[l >> 1].c0 = s.p[l];
      __syncthreads();
    }
  }
  c_store(out[0], &a);
}

static float time_ms(hipEvent_t e0, hipEvent_t e1) {
  float ms = 0;
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  fp_t* io;
  fp12_t *fin, *fout;
  if (hipMalloc((void**)&io, 128 * sizeof(fp_t)) != hipSuccess) return 1;
  if (hipMalloc((void**)&fin, 2 * sizeof(fp12_t)) != hipSuccess) return 1;
  if (hipMalloc((void**)&fout, sizeof(fp12_t)) != hipSuccess) return 1;
  (void)hipMemset(io, 0x11, 128 * sizeof(fp_t));
  (void)hipMemset(fin, 0x01, 2 * sizeof(fp12_t));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const uint32_t N = 2000;
  hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, io, 16u);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, io, N);
  (void)hipEventRecord(e1, 0);
  printf("{\"lone_wave_fp_mul_us\": %.3f,\n", time_ms(e0, e1) * 1e3 / N);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_chain_add, dim3(1), dim3(64), 0, 0, io, N);
  (void)hipEventRecord(e1, 0);
  printf(" \"lone_wave_fp_add_us\": %.4f,\n", time_ms(e0, e1) * 1e3 / N);
  for (uint32_t mode = 0; mode < 2; mode++) {
    hipLaunchKernelGGL(k_cmul, dim3(1), dim3(128), 0, 0, fin, fout, 4u, mode);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_cmul, dim3(1), dim3(128), 0, 0, fin, fout, 500u, mode);
    (void)hipEventRecord(e1, 0);
    printf(" \"c_mul_mode%u_us\": %.3f,\n", mode, time_ms(e0, e1) * 1e3 / 500);
  }
  hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, fin, fout, 2u);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, fin, fout, 20u);
  (void)hipEventRecord(e1, 0);
  printf(" \"fp12_inv_one_lane_us\": %.2f,\n", time_ms(e0, e1) * 1e3 / 20);
  hipLaunchKernelGGL(k_fe, dim3(1), dim3(128), 0, 0, fin, fout, 1u);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_fe, dim3(1), dim3(128), 0, 0, fin, fout, 5u);
  (void)hipEventRecord(e1, 0);
  printf(" \"final_exp_128_lanes_us\": %.1f}\n", time_ms(e0, e1) * 1e3 / 5);
  return 0;
}
