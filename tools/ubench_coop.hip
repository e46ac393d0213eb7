// Latency microbenchmarks of the cooperative building blocks (design study
// for the latency path; not part of the library):
//   * a lone wave's chain of dependent Fp products (the product latency);
//   * c_mul (fp12_coop.h, 128 lanes) in a loop: the latency of one
//     cooperative Fp12 product, and of its rounds taken apart.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_coop tools/ubench_coop.hip
#define BGV_FPMUL_CALL 0
#include "../lodestar_amd/csrc/bgv_internal.h"
#include "../lodestar_amd/csrc/fp12_coop.h"
#include "../lodestar_amd/csrc/coop_g2.h"
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

// one wave, seven 9-lane groups: chains of cooperative G2 doublings / additions
// (coop_g2.h), the latency of one round of the cofactor clearing
__global__ void __launch_bounds__(64) k_cg(const fp12_t* in, fp12_t* out, uint32_t iters, uint32_t add) {
  __shared__ cg_scratch S[CG_GROUPS];
  const uint32_t l = threadIdx.x, g = l / CG_LANES < CG_GROUPS ? l / CG_LANES : CG_GROUPS - 1, r = l - g * CG_LANES;
  const uint32_t s = r < CG_LANES ? r / 3 : 0, q = r < CG_LANES ? r % 3 : 0;
  g2j p, a;
  p.x = in[0].c0.c0;
  p.y = in[0].c0.c1;
  p.z = in[0].c0.c2;
  a.x = in[1].c0.c0;
  a.y = in[1].c0.c1;
  a.z = in[1].c0.c2;
  for (uint32_t k = 0; k < iters; k++) {
    if (add) cg_add(&S[g], s, q, p, p, a);
    else cg_dbl(&S[g], s, q, p, p);
  }
  if (l == 0) {
    out[0].c0.c0 = p.x;
    out[0].c0.c1 = p.y;
    out[0].c0.c2 = p.z;
  }
}

// c_mul's two rounds with clock64() stamps (lane 0 of each wave): t[w][0..5]
// accumulate cycles of R1 operands, R1 product + store, barrier 1, R2 loads,
// R2 add/sub, R2 pulls + sums + store, barrier 2
__global__ void __launch_bounds__(128) k_cmul_t(const fp12_t* in, fp12_t* out, uint32_t iters, unsigned long long* tt) {
  __shared__ cscratch s_;
  __shared__ wfp12 a_, b_;
  c_load(&a_, in[0]);
  c_load(&b_, in[1]);
  BGV_LDS wfp12* a = (BGV_LDS wfp12*)&a_;
  const BGV_LDS wfp12* b = (const BGV_LDS wfp12*)&b_;
  BGV_LDS cscratch* s = (BGV_LDS cscratch*)&s_;
  const uint32_t l = threadIdx.x;
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t it = 0; it < iters; it++) {
    unsigned long long t0 = clock64(), t1 = t0, t2 = t0;
    if (l < 108) {
      const uint32_t p = l / 3, q = l - 3 * p, i = p / 6, j = p - 6 * i;
      fp_t u, v;
      if (q == 0) { u = lds_get(&a->c[i].c0); v = lds_get(&b->c[j].c0); }
      else if (q == 1) { u = lds_get(&a->c[i].c1); v = lds_get(&b->c[j].c1); }
      else fp_add_lazy2(u, lds_get(&a->c[i].c0), lds_get(&a->c[i].c1), v, lds_get(&b->c[j].c0), lds_get(&b->c[j].c1));
      t1 = clock64();
      fp_t r;
      fp_mul(r, u, v);
      lds_put(&s->p[l], r);
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      t2 = clock64();
    }
    __syncthreads();
    const unsigned long long t3 = clock64();
    const uint32_t comp = l >> 6, m = l & 63u;
    const uint32_t k = m / 6 < 6 ? m / 6 : 0u, i = m % 6, j = (k + 6 - i) % 6, pr = i * 6 + j;
    const bool xi = i + j >= 6;
    const fp_t p0 = lds_get(&s->p[3 * pr]), p1 = lds_get(&s->p[3 * pr + 1]), p2 = lds_get(&s->p[3 * pr + 2]);
    fp_t zero;
    fp_set_zero(zero);
    const fp_t& aa = comp ? (xi ? p1 : p0) : p0;
    const fp_t& bb = comp ? p1 : (xi ? p0 : zero);
    fp_t w, t;
    fp_add(w, aa, bb);
    const unsigned long long t4 = clock64();
    fp_sub(t, comp ? p2 : w, comp ? w : (xi ? p2 : p1));
    const unsigned long long t5 = clock64();
    fp_t x = c_pull1(t, (m + 1) & 63u);
    fp_add(t, t, x);
    x = c_pull1(t, (m + 2) & 63u);
    const fp_t y = c_pull1(t, (m + 4) & 63u);
    fp_add(t, t, x);
    fp_add(t, t, y);
    if (m < 36 && i == 0) lds_put(comp ? &a->c[k].c1 : &a->c[k].c0, t);
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t6 = clock64();
    __syncthreads();
    const unsigned long long t7 = clock64();
    acc[0] += t1 - t0; acc[1] += t2 - t1; acc[2] += t3 - t2; acc[3] += t4 - t3; acc[4] += t5 - t4; acc[5] += t6 - t5; acc[6] += t7 - t6;
  }
  if ((l & 63) == 0)
    for (int k = 0; k < 7; k++) tt[(l >> 6) * 8 + k] = acc[k];
  c_store(out[0], &a_);
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
  {
    unsigned long long* tt;
    (void)hipMalloc((void**)&tt, 16 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_cmul_t, dim3(1), dim3(128), 0, 0, fin, fout, 500u, tt);
    unsigned long long h[16];
    (void)hipMemcpy(h, tt, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[7] = {"r1_operands", "r1_product_store", "barrier1", "r2_loads_add", "r2_sub", "r2_pulls_sums_store", "barrier2"};
    for (int w = 0; w < 2; w++) {
      printf(" \"cmul_phase_cycles_wave%d\": {", w);
      for (int k = 0; k < 7; k++) printf("\"%s\": %.0f%s", nm[k], (double)h[w * 8 + k] / 500, k < 6 ? ", " : "},\n");
    }
  }
  for (uint32_t add = 0; add < 2; add++) {
    hipLaunchKernelGGL(k_cg, dim3(1), dim3(64), 0, 0, fin, fout, 4u, add);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_cg, dim3(1), dim3(64), 0, 0, fin, fout, 400u, add);
    (void)hipEventRecord(e1, 0);
    printf(" \"cg_%s_us\": %.3f,\n", add ? "add_6_rounds" : "dbl_3_rounds", time_ms(e0, e1) * 1e3 / 400);
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
