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
#include "fp12_coop.h"

namespace bgv {

#ifndef BGV_TREE_WAVES
#define BGV_TREE_WAVES 2
#endif
#define BGV_TREE_LB __launch_bounds__(64, BGV_TREE_WAVES)

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

// ------------------------------------------- cooperative folds (fp12_coop.h)
#define COOP_LB __launch_bounds__(COOP_THREADS, 2)

// With P pairs per Miller item the item's value sits at offsets P t of the job
// and every other entry is 1 (k_miller, k_miller_kv), so the folds step over
// the items only: at C4 that cuts the per-job chain from 98 to 49 (P = 2) or
// 25 (P = 4) Fp12 products.
__device__ __forceinline__ static uint32_t fold_step(const dev_batch& b) { return b.pairs_per_item ? b.pairs_per_item : 1u; }

// first level of the two-level fold (few large jobs, e.g. one 64-set gossip
// batch, and the C4 segment's 98-set blocks): workgroup (g, j) folds the job's
// values in [beg + G g, beg + G g + G) into f_set[beg + G g] (in place: all
// reads precede the one write, and the groups are disjoint); k_job_fold then
// walks the job with stride G
__global__ void COOP_LB k_job_prefold(dev_batch b, dev_work w) {
  __shared__ cscratch s;
  __shared__ wfp12 acc, x;
  const uint32_t j = blockIdx.y, G = 1u << b.prefold_log2;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  const uint32_t g0 = beg + blockIdx.x * G;
  if (w.job_code[j] != C_OK || g0 + 1 >= end) return;  // uniform per workgroup
  const uint32_t g1 = min(end, g0 + G);
  c_load(&acc, w.f_set[g0]);
  for (uint32_t i = g0 + fold_step(b); i < g1; i += fold_step(b)) {
    c_load(&x, w.f_set[i]);
    c_mul(&acc, &acc, &x, &s);
  }
  c_store(w.f_set[g0], &acc);
}

// one workgroup per job: f_job = (job pair value) * prod of the job's set
// values (or of its group values after k_job_prefold, stride > 1), folded in
// order at the latency of one Fp product per step
__global__ void COOP_LB k_job_fold(dev_batch b, dev_work w, uint32_t stride) {
  __shared__ cscratch s;
  __shared__ wfp12 acc, x;
  const uint32_t j = blockIdx.x;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  if (w.job_code[j] != C_OK) {
    c_set_one(&acc);  // rejected jobs take no part in the batch product
  } else {
    c_load(&acc, w.f_set[b.n_sets + j]);
    for (uint32_t i = beg; i < end; i += stride) {
      c_load(&x, w.f_set[i]);
      c_mul(&acc, &acc, &x, &s);
    }
  }
  c_store(w.f_job[j], &acc);
  c_store(w.f_batch[j], &acc);
}

// workgroup g: dst[g] = prod src[F g .. min(n, F g + F)) with fan-in F; with
// one workgroup dst may alias src (every read precedes the write).  A
// fan-in of 8 keeps the chain of sequential Fp12 products short: 1,024 job
// values fold in 8 + 8 + 8 + 8 + 2 products instead of 32 + 32.
constexpr uint32_t FOLD_FAN = 8;
__global__ void COOP_LB k_fold(const fp12_t* src, uint32_t n, fp12_t* dst) {
  __shared__ cscratch s;
  __shared__ wfp12 acc, x;
  const uint32_t beg = blockIdx.x * FOLD_FAN, end = min(n, beg + FOLD_FAN);
  c_load(&acc, src[beg]);
  for (uint32_t i = beg + 1; i < end; i++) {
    c_load(&x, src[i]);
    c_mul(&acc, &acc, &x, &s);
  }
  c_store(dst[blockIdx.x], &acc);
}

// the whole-batch check: ONE final exponentiation over 128 lanes
__global__ void COOP_LB k_batch_final(dev_batch b, dev_work w) {
  __shared__ cscratch s;
  if (b.n_jobs == 0) {
    if (threadIdx.x == 0) w.flags[0] = 0u;
    return;
  }
  const bool one = c_final_exp_is_one(w.f_batch[0], &s);
  if (threadIdx.x == 0) w.flags[0] = one ? 1u : 0u;
}

// per-job verdicts; a final exponentiation per job only when the batch check
// failed (the worker's per-job retry, multithread/worker.ts:74-85), one
// workgroup per job
__global__ void COOP_LB k_job_final(dev_batch b, dev_work w) {
  __shared__ cscratch s;
  const uint32_t j = blockIdx.x;
  const int32_t code = w.job_code[j];
  int32_t res;
  if (code != C_OK) {
    res = -code;
  } else if (w.flags[0]) {
    res = 1;  // whole batch verified: every job is valid
  } else {
    res = c_final_exp_is_one(w.f_job[j], &s) ? 1 : 0;
  }
  if (threadIdx.x == 0) w.job_result[j] = res;
}

// ------------------------------------------------- multi-GPU combination
__global__ void COOP_LB k_combine_final(const fp12_t* parts, uint32_t n, uint32_t* flag) {
  __shared__ cscratch s;
  __shared__ wfp12 acc, x;
  __shared__ fp12_t g;
  c_set_one(&acc);
  for (uint32_t k = 0; k < n; k++) {
    c_load(&x, parts[k]);
    c_mul(&acc, &acc, &x, &s);
  }
  c_store(g, &acc);
  const bool one = c_final_exp_is_one(g, &s);
  if (threadIdx.x == 0) flag[0] = one ? 1u : 0u;
}

// bgv_debug_stages: out[i] = FE(in[i]) (the cubed value of c_final_exp), one
// cooperative workgroup per element
__global__ void COOP_LB k_final_exp_many(const fp12_t* in, fp12_t* out) {
  __shared__ cscratch s;
  __shared__ fp12_t r;
  c_final_exp(&r, in[blockIdx.x], &s);
  if (threadIdx.x == 0) out[blockIdx.x] = r;
}

#undef gtid

void launch_fp12_tail(hipStream_t st, int stage, const dev_batch& b, const dev_work& w) {
  const uint32_t span = 1u << b.span_log2;
  auto grid = [](uint32_t n) { return dim3((n + 63u) / 64u); };
  const dim3 ct(COOP_THREADS);
  if (stage == ST_F_TREE) {
    if (!b.n_jobs) return;
    if (span <= 256) {  // every job folds in one workgroup
      uint32_t stride = b.pairs_per_item ? b.pairs_per_item : 1u;  // fold_step
      if (b.prefold_log2) {  // few large jobs: fold groups side by side first
        stride = 1u << b.prefold_log2;
        hipLaunchKernelGGL(k_job_prefold, dim3((span + stride - 1) / stride, b.n_jobs), ct, 0, st, b, w);
      }
      hipLaunchKernelGGL(k_job_fold, dim3(b.n_jobs), ct, 0, st, b, w, stride);
      return;
    }
    // larger jobs: segmented pairwise tree first
    if (b.n_sets)
      for (uint32_t s = 1; s < span; s *= 2) hipLaunchKernelGGL(k_f_level, grid(b.n_sets), dim3(64), 0, st, b, w, s);
    hipLaunchKernelGGL(k_job_f, grid(b.n_jobs), dim3(64), 0, st, b, w, span);
  } else if (stage == ST_BATCH_PROD) {
    // fold by FOLD_FAN, ping-ponging f_batch <-> f_tmp, the product landing in f_batch[0]
    uint32_t n = b.n_jobs;
    fp12_t* src = w.f_batch;
    while (n > FOLD_FAN) {
      fp12_t* dst = src == w.f_batch ? w.f_tmp : w.f_batch;
      const uint32_t groups = (n + FOLD_FAN - 1) / FOLD_FAN;
      hipLaunchKernelGGL(k_fold, dim3(groups), ct, 0, st, src, n, dst);
      src = dst;
      n = groups;
    }
    if (n > 1 || (n == 1 && src != w.f_batch)) hipLaunchKernelGGL(k_fold, dim3(1), ct, 0, st, src, n, w.f_batch);
  } else if (stage == ST_BATCH_FINAL) {
    hipLaunchKernelGGL(k_batch_final, dim3(1), ct, 0, st, b, w);
  } else if (stage == ST_JOB_FINAL) {
    if (b.n_jobs) hipLaunchKernelGGL(k_job_final, dim3(b.n_jobs), ct, 0, st, b, w);
  }
}

void launch_final_exp_many(hipStream_t st, const fp12_t* in, fp12_t* out, uint32_t n) {
  if (n) hipLaunchKernelGGL(k_final_exp_many, dim3(n), dim3(COOP_THREADS), 0, st, in, out);
}

void launch_combine_final(hipStream_t st, const fp12_t* parts, uint32_t n, uint32_t* flag) {
  hipLaunchKernelGGL(k_combine_final, dim3(1), dim3(COOP_THREADS), 0, st, parts, n, flag);
}

}  // namespace bgv
