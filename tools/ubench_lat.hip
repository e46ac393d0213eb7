// Latency microbenchmarks of the non-product building blocks of the
// cooperative (latency-mode) kernels: a lone wave's dependent chains of Fp
// additions in several carry schemes, and the cost of one LDS exchange round
// with and without a workgroup barrier.  Design study, not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_lat tools/ubench_lat.hip
#define BGV_FPMUL_CALL 0
#include "../lodestar_amd/csrc/bgv_internal.h"
#include "../lodestar_amd/csrc/lds.h"
#include <stdio.h>

using namespace bgv;

// carry-select: the high six limbs are summed for both carries in parallel
__device__ __forceinline__ void fp_add_cs(fp_t& r, const fp_t& a, const fp_t& b) {
  uint32_t s[NL], h1[6], t[NL], u1[6];
  uint32_t c = 0, c0 = 0, c1 = 1;
#pragma unroll
  for (int i = 0; i < 6; i++) s[i] = addc32(a.l[i], b.l[i], c, c);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    s[6 + i] = addc32(a.l[6 + i], b.l[6 + i], c0, c0);
    h1[i] = addc32(a.l[6 + i], b.l[6 + i], c1, c1);
  }
  const uint32_t mc = 0u - c;
#pragma unroll
  for (int i = 0; i < 6; i++) s[6 + i] = (h1[i] & mc) | (s[6 + i] & ~mc);
  uint32_t bw = 0, b0 = 0, b1 = 1;
#pragma unroll
  for (int i = 0; i < 6; i++) t[i] = subb32(s[i], P_MOD.l[i], bw, bw);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    t[6 + i] = subb32(s[6 + i], P_MOD.l[6 + i], b0, b0);
    u1[i] = subb32(s[6 + i], P_MOD.l[6 + i], b1, b1);
  }
  const uint32_t mb = 0u - bw;
  const uint32_t neg = (b1 & bw) | (b0 & ~bw & 1u);  // borrow out of the full subtraction
  const uint32_t keep = 0u - neg;
#pragma unroll
  for (int i = 0; i < 6; i++) t[6 + i] = (u1[i] & mb) | (t[6 + i] & ~mb);
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (s[i] & keep) | (t[i] & ~keep);
}

// four-way split of the carry chains (three-limb blocks)
__device__ __forceinline__ void fp_add_cs4(fp_t& r, const fp_t& a, const fp_t& b) {
  uint32_t s0[NL], s1[NL], t0[NL], t1[NL];
  uint32_t cb0[4], cb1[4], bb0[4], bb1[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t x = 0, y = 1;
#pragma unroll
    for (int i = 3 * k; i < 3 * k + 3; i++) {
      s0[i] = addc32(a.l[i], b.l[i], x, x);
      s1[i] = addc32(a.l[i], b.l[i], y, y);
    }
    cb0[k] = x;
    cb1[k] = y;
  }
  uint32_t s[NL];
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t m = 0u - c;
#pragma unroll
    for (int i = 3 * k; i < 3 * k + 3; i++) s[i] = (s1[i] & m) | (s0[i] & ~m);
    c = (cb1[k] & c) | (cb0[k] & (c ^ 1u));
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t x = 0, y = 1;
#pragma unroll
    for (int i = 3 * k; i < 3 * k + 3; i++) {
      t0[i] = subb32(s[i], P_MOD.l[i], x, x);
      t1[i] = subb32(s[i], P_MOD.l[i], y, y);
    }
    bb0[k] = x;
    bb1[k] = y;
  }
  uint32_t t[NL];
  uint32_t bw = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t m = 0u - bw;
#pragma unroll
    for (int i = 3 * k; i < 3 * k + 3; i++) t[i] = (t1[i] & m) | (t0[i] & ~m);
    bw = (bb1[k] & bw) | (bb0[k] & (bw ^ 1u));
  }
  const uint32_t keep = 0u - bw;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (s[i] & keep) | (t[i] & ~keep);
}

template <int V>
__global__ void __launch_bounds__(64) k_add(fp_t* io, uint32_t iters) {
  fp_t x = io[threadIdx.x], y = io[64 + threadIdx.x];
  for (uint32_t k = 0; k < iters; k++) {
    if (V == 0) fp_add(x, x, y);
    else if (V == 1) fp_add_cs(x, x, y);
    else if (V == 2) fp_add_cs4(x, x, y);
    else fp_sub(x, x, y);
  }
  io[threadIdx.x] = x;
}

// one exchange round: lanes < 9 form a product, write it to LDS, the barrier,
// then every lane reads its neighbour's value (mode 0: __syncthreads, mode 1:
// wave-level only (64 threads), mode 2: no product, barrier + LDS only)
template <int MODE>
__global__ void __launch_bounds__(64) k_round(fp_t* io, uint32_t iters) {
  __shared__ fp_t buf[64];
  const uint32_t l = threadIdx.x;
  fp_t x = io[l], y = io[64 + l];
  for (uint32_t k = 0; k < iters; k++) {
    if (MODE != 2 && l < 9) fp_mul(x, x, y);
    lds_put((BGV_LDS fp_t*)&buf[l], x);
    if (MODE == 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
      __syncthreads();
    }
    x = lds_get((BGV_LDS fp_t*)&buf[(l + 1) & 63]);
    if (MODE == 1) {
      __builtin_amdgcn_wave_barrier();
    } else {
      __syncthreads();
    }
  }
  io[l] = x;
}

static float time_ms(hipEvent_t e0, hipEvent_t e1) {
  float ms = 0;
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

template <class K>
static double run_us(K kern, fp_t* io, uint32_t n) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, 16u);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, n);
  (void)hipEventRecord(e1, 0);
  const double us = time_ms(e0, e1) * 1e3 / n;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return us;
}

int main() {
  fp_t* io;
  if (hipMalloc((void**)&io, 128 * sizeof(fp_t)) != hipSuccess) return 1;
  (void)hipMemset(io, 0x05, 128 * sizeof(fp_t));
  const uint32_t N = 4000;
  printf("{\"fp_add_us\": %.4f, ", run_us(k_add<0>, io, N));
  printf("\"fp_add_carry_select2_us\": %.4f, ", run_us(k_add<1>, io, N));
  printf("\"fp_add_carry_select4_us\": %.4f, ", run_us(k_add<2>, io, N));
  printf("\"fp_sub_us\": %.4f, ", run_us(k_add<3>, io, N));
  printf("\"round_mul_syncthreads_us\": %.4f, ", run_us(k_round<0>, io, N / 4));
  printf("\"round_mul_wave_us\": %.4f, ", run_us(k_round<1>, io, N / 4));
  printf("\"round_lds_sync_only_us\": %.4f}\n", run_us(k_round<2>, io, N));
  return 0;
}
