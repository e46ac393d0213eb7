// Fp12 tail of the batch verifier: the product trees (ST_F_TREE,
// ST_BATCH_PROD), the final exponentiations (ST_BATCH_FINAL, ST_JOB_FINAL)
// and the multi-GPU combination.
//
// A separate translation unit because it wants the opposite code generation
// to bgv_kernels.hip: these kernels are latency-bound (log2 levels, few lanes
// per level after the first, one wave for the final exponentiation) and run
// fastest with the Fp product inlined into the non-inlined Fp2 routines
// (BGV_FPMUL_CALL=0): k_f_level x7 + k_job_f take 3.2 ms at C4 this way
// against 5.1 ms with the register-ABI leaf.
#ifndef BGV_FPMUL_CALL
#define BGV_FPMUL_CALL 0
#endif
#include "bgv_internal.h"
#include "fp12_wave.h"

namespace bgv {

#ifndef BGV_TREE_WAVES
#define BGV_TREE_WAVES 2
#endif
#define BGV_TREE_LB __launch_bounds__(64, BGV_TREE_WAVES)
#define BGV_BULK BGV_TREE_LB

__device__ __forceinline__ static uint32_t tree_gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }
#define gtid tree_gtid

// per-job product of the Miller values: segmented pairwise tree over the
// job's sets (level s multiplies f[i] by f[i + s] for i = beg + 2s k), then
// k_job_f folds the span-strided survivors and the job's (-G1, S_job) value
__global__ void BGV_TREE_LB k_f_level(dev_batch b, dev_work w, uint32_t s) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const uint32_t j = w.set_job[i];
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  if (((i - beg) % (2 * s)) != 0 || i + s >= end) return;
  fp12_t a = w.f_set[i];
  fp12_mul(a, a, w.f_set[i + s]);
  w.f_set[i] = a;
}

__global__ void BGV_TREE_LB k_job_f(dev_batch b, dev_work w, uint32_t span) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  fp12_t f;
  if (w.job_code[j] != C_OK) {
    fp12_one(f);  // rejected jobs take no part in the batch product
  } else {
    f = w.f_set[beg];
    for (uint32_t i = beg + span; i < end; i += span) fp12_mul(f, f, w.f_set[i]);
    fp12_mul(f, f, w.f_set[b.n_sets + j]);
  }
  w.f_job[j] = f;
  w.f_batch[j] = f;
}

// ---------------------------------------------------------- batch product
__global__ void BGV_TREE_LB k_batch_level(dev_batch b, dev_work w, uint32_t s) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs || (j % (2 * s)) != 0 || j + s >= b.n_jobs) return;
  fp12_t a = w.f_batch[j];
  fp12_mul(a, a, w.f_batch[j + s]);
  w.f_batch[j] = a;
}

// the whole-batch check: ONE final exponentiation, wave-cooperative (fp12_wave.h)
__global__ void BGV_BULK k_batch_final(dev_batch b, dev_work w) {
  __shared__ wscratch s;
  if (b.n_jobs == 0) {
    if (threadIdx.x == 0) w.flags[0] = 0u;
    return;
  }
  const bool one = w_final_exp_is_one(w.f_batch[0], &s);
  if (threadIdx.x == 0) w.flags[0] = one ? 1u : 0u;
}

// ------------------------------------------------------------ k_job_final
__global__ void BGV_BULK k_job_final(dev_batch b, dev_work w) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  const int32_t code = w.job_code[j];
  int32_t res;
  if (code != C_OK) {
    res = -code;
  } else if (w.flags[0]) {
    res = 1;  // whole batch verified: every job is valid
  } else {
    fp12_t r;
    fp12_final_exp(r, w.f_job[j]);
    res = fp12_is_one(r) ? 1 : 0;
  }
  w.job_result[j] = res;
}

// ------------------------------------------------- multi-GPU combination
__global__ void BGV_BULK k_combine_final(const fp12_t* parts, uint32_t n, uint32_t* flag) {
  __shared__ wscratch s;
  __shared__ fp12_t g;
  if (threadIdx.x == 0) {
    fp12_one(g);
    for (uint32_t k = 0; k < n; k++) fp12_mul(g, g, parts[k]);
  }
  __syncthreads();
  const bool one = w_final_exp_is_one(g, &s);
  if (threadIdx.x == 0) flag[0] = one ? 1u : 0u;
}

#undef gtid

void launch_fp12_tail(hipStream_t st, int stage, const dev_batch& b, const dev_work& w) {
  const uint32_t span = 1u << b.span_log2;
  auto grid = [](uint32_t n) { return dim3((n + 63u) / 64u); };
  if (stage == ST_F_TREE) {
    if (b.n_sets)
      for (uint32_t s = 1; s < span; s *= 2) hipLaunchKernelGGL(k_f_level, grid(b.n_sets), dim3(64), 0, st, b, w, s);
    if (b.n_jobs) hipLaunchKernelGGL(k_job_f, grid(b.n_jobs), dim3(64), 0, st, b, w, span);
  } else if (stage == ST_BATCH_PROD) {
    for (uint32_t s = 1; s < b.n_jobs; s *= 2) hipLaunchKernelGGL(k_batch_level, grid(b.n_jobs), dim3(64), 0, st, b, w, s);
  } else if (stage == ST_BATCH_FINAL) {
    hipLaunchKernelGGL(k_batch_final, dim3(1), dim3(64), 0, st, b, w);
  } else if (stage == ST_JOB_FINAL) {
    if (b.n_jobs) hipLaunchKernelGGL(k_job_final, grid(b.n_jobs), dim3(64), 0, st, b, w);
  }
}

void launch_combine_final(hipStream_t st, const fp12_t* parts, uint32_t n, uint32_t* flag) {
  hipLaunchKernelGGL(k_combine_final, dim3(1), dim3(64), 0, st, parts, n, flag);
}

}  // namespace bgv
