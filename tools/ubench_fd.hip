// Design study (not part of the library): the Fp product on 12 x 32-bit
// limbs (fp.h, the library's register-ABI leaf) against a signed 14 x 28-bit
// digit form that stays unpacked between products (no unpack/pack, no final
// subtraction, carry-free additions).  Lone-wave latency and full-chip
// throughput of a chain of Fp products and of a chain of Karatsuba Fp2
// products (3 products + the additions of each form).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_fd tools/ubench_fd.hip && ./tools/ubench_fd
#define BGV_FPMUL_CALL 1
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../lodestar_amd/csrc/fp2.h"

namespace bgv {

constexpr int ND = 14;
typedef int32_t fd_vec_t __attribute__((ext_vector_type(14)));

// signed product scanning, Montgomery reduction by 2^28 per digit (R = 2^392)
static __device__ __noinline__ fd_vec_t fd_mul_leaf(fd_vec_t a, fd_vec_t b) {
  uint64_t acc[2 * ND];
#pragma unroll
  for (int k = 0; k < 2 * ND; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < ND; i++)
#pragma unroll
    for (int j = 0; j < ND; j++) acc[i + j] += (uint64_t)((int64_t)a[i] * (int64_t)b[j]);
#pragma unroll
  for (int i = 0; i < ND; i++) {
    const uint32_t m = ((uint32_t)acc[i] * P28_INV) & M28;
#pragma unroll
    for (int j = 0; j < ND; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += (uint64_t)((int64_t)acc[i] >> 28);
  }
  fd_vec_t r;
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < ND - 1; k++) {
    const int64_t v = (int64_t)acc[ND + k] + c;
    r[k] = (int32_t)(v & M28);
    c = v >> 28;
  }
  r[ND - 1] = (int32_t)((int64_t)acc[2 * ND - 1] + c);
  return r;
}

__device__ __forceinline__ fd_vec_t fd_norm(fd_vec_t a) {
  fd_vec_t t;
  t[0] = a[0] & (int32_t)M28;
#pragma unroll
  for (int k = 1; k < ND - 1; k++) t[k] = (a[k] & (int32_t)M28) + (a[k - 1] >> 28);
  t[ND - 1] = a[ND - 1] + (a[ND - 2] >> 28);
  return t;
}

}  // namespace bgv

using namespace bgv;

__global__ void __launch_bounds__(64) k_fp_chain(fp_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp_t x = io[2 * i], y = io[2 * i + 1];
  for (uint32_t t = 0; t < iters; t++) fp_mul(x, x, y);
  io[2 * i] = x;
}

__global__ void __launch_bounds__(64) k_fd_chain(fd_vec_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fd_vec_t x = io[2 * i], y = io[2 * i + 1];
  for (uint32_t t = 0; t < iters; t++) x = fd_mul_leaf(x, y);
  io[2 * i] = x;
}

__global__ void __launch_bounds__(64) k_fp2_chain(fp2_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fp2_t x = io[2 * i], y = io[2 * i + 1];
  for (uint32_t t = 0; t < iters; t++) fp2_mul_inl(x, x, y);
  io[2 * i] = x;
}

// Karatsuba over the digit form: sums digit-wise, c1 normalised (its three
// terms would otherwise grow the next product's digit bound)
__global__ void __launch_bounds__(64) k_fd2_chain(fd_vec_t* io, uint32_t iters) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  fd_vec_t x0 = io[4 * i], x1 = io[4 * i + 1], y0 = io[4 * i + 2], y1 = io[4 * i + 3];
  for (uint32_t t = 0; t < iters; t++) {
    const fd_vec_t t0 = fd_mul_leaf(x0, y0), t1 = fd_mul_leaf(x1, y1), t2 = fd_mul_leaf(x0 + x1, y0 + y1);
    x0 = t0 - t1;
    x1 = fd_norm(t2 - t0 - t1);
  }
  io[4 * i] = x0;
  io[4 * i + 1] = x1;
}

template <class T>
static float run(void (*k)(T*, uint32_t), T* d, uint32_t blocks, uint32_t iters) {
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
  void* d;
  hipMalloc(&d, (size_t)big * 64 * 4 * 64);
  hipMemset(d, 0x11, (size_t)big * 64 * 4 * 64);
  const uint32_t it = 2000;
  struct { const char* name; float lone, thr; int per; } r[4];
  r[0] = {"fp_mul chain", run(k_fp_chain, (fp_t*)d, 1, it), run(k_fp_chain, (fp_t*)d, big, it / 10), 1};
  r[1] = {"fd_mul chain", run(k_fd_chain, (fd_vec_t*)d, 1, it), run(k_fd_chain, (fd_vec_t*)d, big, it / 10), 1};
  r[2] = {"fp2_mul chain", run(k_fp2_chain, (fp2_t*)d, 1, it), run(k_fp2_chain, (fp2_t*)d, big, it / 10), 3};
  r[3] = {"fd2_mul chain", run(k_fd2_chain, (fd_vec_t*)d, 1, it), run(k_fd2_chain, (fd_vec_t*)d, big, it / 10), 3};
  printf("{");
  for (int k = 0; k < 4; k++) {
    const double lone_us = r[k].lone * 1e3 / it;
    const double thr = (double)big * 64 * (it / 10) * r[k].per / (r[k].thr * 1e-3) / 1e9;
    printf("%s\"%s\": {\"lone_wave_us_per_step\": %.4f, \"chip_G_fpmul_per_s\": %.2f}", k ? ", " : "", r[k].name, lone_us, thr);
  }
  printf("}\n");
  return 0;
}
