// The set-pair Miller loop kernel (k_miller), in its own translation unit:
// it runs at 1 wave/SIMD (512-register budget, spills in AGPRs) with its Fp12
// accumulator in LDS, which no other kernel of bgv_kernels.hip wants.
// Work items: every job's sets taken pairs_per_item (1, 2 or 4) at a time (one
// shared Fp12 accumulator and squaring per item: miller_loop2 /
// miller_loop_lines / miller_loop_lines4), then one item per job for its
// (-G1, S_job) pair.  Item offsets per job come from a scan
// (bgv_kernels.hip k_item_count / k_item_job).
#ifndef BGV_FPMUL_CALL
#ifdef BGV_MILLER_FPMUL_CALL
#define BGV_FPMUL_CALL BGV_MILLER_FPMUL_CALL
#else
#define BGV_FPMUL_CALL 1
#endif
#endif
#ifndef BGV_FP2_INLINE
#define BGV_FP2_INLINE 1
#endif
#ifndef BGV_FP6_INLINE
#define BGV_FP6_INLINE 1
#endif
#ifndef BGV_POINT_INLINE
#define BGV_POINT_INLINE 1  // jac_dbl / jac_add / jac_add_aff: 2049k -> 2155k sets/s
#endif
#ifndef BGV_MILLER_WAVES
#define BGV_MILLER_WAVES 1
#endif
#ifndef BGV_MILLER_LDS_F
#define BGV_MILLER_LDS_F 1
#endif
// per-unit inlining knobs (A/B builds): Fp12 layer and Miller steps.  The
// Fp12 layer is inlined into the loops: a non-inlined fp12_sqr saved and
// restored ~1.2 KB of callee-saved registers through scratch on every call
// (k_miller: 11.2 GB FETCH + WRITE per C4 launch, profiles/r03_pmc_*.csv);
// same-box A/B at C4: 39.04 / 38.82 -> 38.55 / 38.32 ms (r03)
#ifndef BGV_MILLER_FP12_INLINE
#define BGV_MILLER_FP12_INLINE 1
#endif
#if BGV_MILLER_FP12_INLINE
#define BGV_FP12_INLINE BGV_MILLER_FP12_INLINE
#endif
#ifdef BGV_MILLER_STEP_INLINE
#define BGV_STEP_INLINE BGV_MILLER_STEP_INLINE
#endif
#include "bgv_internal.h"
#include "miller_duo.h"
#include "miller_quad.h"
#include "miller_kv.h"

namespace bgv {

__global__ void __launch_bounds__(64, BGV_MILLER_WAVES) k_miller(dev_batch b, dev_work w, uint32_t jobs_part) {
  const uint32_t n_items = w.item_off[b.n_jobs];
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) + (jobs_part ? n_items : 0u);
  if (jobs_part ? t >= n_items + b.n_jobs : t >= n_items) return;
  // the accumulator lives in LDS: at 1 wave/SIMD a lane has 640 B of it, and
  // every fp12_sqr / fp12_mul_line call reads and writes f by reference, which
  // from a stack slot would be ~3 KB of scratch traffic per lane per bit
#if BGV_MILLER_LDS_F
  __shared__ fp12_t f_lds[64];
  fp12_t& f = f_lds[threadIdx.x];
#else
  fp12_t f;
#endif
  if (t < n_items) {
    const uint32_t j = w.item_job[t];
    const uint32_t i1 = b.job_off[j] + b.pairs_per_item * (t - w.item_off[j]);
    const uint32_t cnt = min(b.pairs_per_item, b.job_off[j + 1] - i1);  // live pairs of the item (1..4)
    const bool two = b.pairs_per_item == 2 && cnt == 2;
    bool ok = true;
    for (uint32_t k = 0; k < cnt; k++) ok &= w.pk_code[i1 + k] == C_OK;
    // a parse error rejects the whole job, so its Miller values are never used;
    // signature codes are not known yet (this part overlaps ST_SIG_SCALE)
    if (!ok) fp12_one(f);
    else if (b.pairs_per_item == 4) {
      // dead pairs (cnt < 4) read a live set's line and P; their lines are forced to 1
      const uint32_t q1 = cnt > 1 ? i1 + 1 : i1, q2 = cnt > 2 ? i1 + 2 : i1, q3 = cnt > 3 ? i1 + 3 : i1;
      miller_loop_lines4(f, w.lines, b.n_sets, w.rpk_aff[i1], w.rpk_aff[q1], w.rpk_aff[q2], w.rpk_aff[q3], i1, q1, q2, q3, cnt);
    } else if (b.lines) miller_loop_lines(f, w.lines, b.n_sets, w.rpk_aff[i1], i1, w.rpk_aff[two ? i1 + 1 : i1], i1 + 1, two);
    else if (two) miller_loop2(f, w.rpk_aff[i1], w.h_aff[i1], w.rpk_aff[i1 + 1], w.h_aff[i1 + 1]);
    else miller_loop(f, w.rpk_aff[i1], false, w.h_aff[i1], false);
    w.f_set[i1] = f;
    if (cnt > 1) {
      fp12_one(f);
      for (uint32_t k = 1; k < cnt; k++) w.f_set[i1 + k] = f;
    }
  } else {
    const uint32_t j = t - n_items;
    g1a ng;
    ng.x = G1_X_MONT;
    ng.y = G1_NEG_Y_MONT;
    if (w.job_code[j] != C_OK || w.s_inf[j]) fp12_one(f);
    else miller_loop(f, ng, false, w.s_aff[j], false);
    w.f_set[b.n_sets + j] = f;
  }
}

// Two lanes per pair (miller_duo.h), 32 pairs per wave: pair t < n_sets is
// (r_t PK_t, H(m_t)); a pair whose pubkey was rejected contributes 1.  For
// batches between the cooperative layouts' reach and the one-lane loop's
// (prepare(): ~6,000 to 35,000 sets), where one lane per pair leaves most
// SIMDs idle and six lanes per pair oversubscribe them.
__global__ void __launch_bounds__(64, 1) k_miller_duo(dev_batch b, dev_work w, uint32_t count) {
  __shared__ duo_x_t sx[32];
  const uint32_t lane = threadIdx.x, pr = lane >> 1, h = lane & 1u;
  const uint32_t t = blockIdx.x * 32u + pr;
  if (t >= count) return;  // both lanes of a pair leave together
  if (w.pk_code[t] != C_OK) {  // rejected job: its Miller values are never used
    fp6_t v;
    if (h) fp6_zero(v);
    else fp6_one(v);
    if (h) w.f_set[t].c1 = v;
    else w.f_set[t].c0 = v;
    return;
  }
  const g1a P = w.rpk_aff[t];
  const g2a Q = w.h_aff[t];
  fp6_t fh;
  duo_miller(fh, P, Q, h, sx[pr]);
  if (h) w.f_set[t].c1 = fh;
  else w.f_set[t].c0 = fh;
}

void launch_miller_duo(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_sets) hipLaunchKernelGGL(k_miller_duo, dim3((b.n_sets + 31u) / 32u), dim3(64), 0, st, b, w, b.n_sets);
}

// Four lanes per pair (miller_quad.h), 16 pairs per wave: the layout for
// batches of ~6,000 to ~25,000 sets (prepare()), where two lanes per pair
// leave most SIMDs idle and the cooperative six-lane layout oversubscribes
// them at three times the per-iteration work.
__global__ void __launch_bounds__(64, 1) k_miller_quad(dev_batch b, dev_work w, uint32_t count) {
  __shared__ quad_x_t sx[16];
  __shared__ fp2_t zs;  // the zero operand (miller_quad.h address selects)
  const uint32_t lane = threadIdx.x, pr = lane >> 2, h = (lane >> 1) & 1u, s = lane & 1u;
  const uint32_t t = blockIdx.x * 16u + pr;
  zs = fp2_zero();  // every lane stores the same value; the wave's first read follows it in issue order
  coop_wave_sync();
  if (t >= count) return;  // the four lanes of a pair leave together
  if (w.pk_code[t] != C_OK) {  // rejected job: its Miller values are never used
    if (s == 0) {
      fp6_t v;
      if (h) fp6_zero(v);
      else fp6_one(v);
      if (h) w.f_set[t].c1 = v;
      else w.f_set[t].c0 = v;
    }
    return;
  }
  const g1a P = w.rpk_aff[t];
  const g2a Q = w.h_aff[t];
  fp6_t fh;
  quad_miller(fh, P, Q, h, s, sx[pr], &zs);
  if (s == 0) {
    if (h) w.f_set[t].c1 = fh;
    else w.f_set[t].c0 = fh;
  }
}

void launch_miller_quad(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_sets) hipLaunchKernelGGL(k_miller_quad, dim3((b.n_sets + 15u) / 16u), dim3(64), 0, st, b, w, b.n_sets);
}

// Two pairs per group of 3 S lanes in Karatsuba views (miller_kv.h): the
// work items of k_miller (a job's sets two at a time, item_off / item_job),
// f_set[i1] = f_{x,Q1}(P1) f_{x,Q2}(P2) and f_set[i1 + 1] = 1 (as k_miller)
template <int S>
__global__ void __launch_bounds__(64, 1) k_miller_kv(dev_batch b, dev_work w) {
  constexpr int LANES = 3 * S, G = 64 / LANES;
  __shared__ mkv_scratch sm[G + 1];
  const uint32_t lane = threadIdx.x, grp = lane / LANES, r = lane % LANES, s = r / 3u, q = r % 3u;
  const uint32_t n_items = w.item_off[b.n_jobs];
  if (n_items == 0) return;  // wave-uniform: a batch of empty jobs has no item (item_job[0] is stale)
  const uint32_t t0 = blockIdx.x * G + grp;
  const bool own = grp < (uint32_t)G && t0 < n_items;
  const uint32_t t = own ? t0 : 0u;
  const mkv_grp<S> g{&sm[grp], s, q};
  if (s == 0 && q == 0) {
    fp_t z;
    fp_set_zero(z);
    lds_put(&((BGV_LDS mkv_scratch*)g.sc)->Z, z);
  }
  coop_wave_sync();
  const uint32_t j = w.item_job[t];
  const uint32_t i1 = b.job_off[j] + 2u * (t - w.item_off[j]);
  const bool two = i1 + 1u < b.job_off[j + 1];
  const uint32_t idx[2] = {i1, two ? i1 + 1u : i1};
  mkv_pair T[2];
  fp_t qx[2], qy[2];
  const fp_t one = mkv_one(q);
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const g1a P = w.rpk_aff[idx[p]];
    const g2a Q = w.h_aff[idx[p]];
    qx[p] = kv_view(Q.x, q);
    qy[p] = kv_view(Q.y, q);
    T[p].x = qx[p];
    T[p].y = qy[p];
    T[p].z = one;
    T[p].xp = P.x;
    T[p].yp = P.y;
  }
  fp_t fa[3], fb[3];
  mkv_miller2<S>(g, T, qx, qy, two, fa, fb);
  if (!own || s != 0 || q > 1) return;
  // a rejected pubkey rejects the job: its Miller values are never used (1, as k_miller)
  const bool ok = w.pk_code[i1] == C_OK && (!two || w.pk_code[i1 + 1u] == C_OK);
  // views 0 and 1 are the components: each of the two lanes writes its own
  fp12_t* f = &w.f_set[i1];
  fp2_t* cs[6] = {&f->c0.c0, &f->c0.c1, &f->c0.c2, &f->c1.c0, &f->c1.c1, &f->c1.c2};
  const fp_t* vs[6] = {&fa[0], &fa[1], &fa[2], &fb[0], &fb[1], &fb[2]};
  fp_t z;
  fp_set_zero(z);
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const fp_t v = ok ? *vs[k] : ((k == 0 && q == 0) ? FP_ONE : z);
    if (q) cs[k]->c1 = v;
    else cs[k]->c0 = v;
  }
  if (two) {
    fp12_t* f2 = &w.f_set[i1 + 1u];
    fp2_t* ds[6] = {&f2->c0.c0, &f2->c0.c1, &f2->c0.c2, &f2->c1.c0, &f2->c1.c1, &f2->c1.c2};
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const fp_t v = (k == 0 && q == 0) ? FP_ONE : z;
      if (q) ds[k]->c1 = v;
      else ds[k]->c0 = v;
    }
  }
}

void launch_miller_kv(hipStream_t st, const dev_batch& b, const dev_work& w) {
  // items <= n_sets / 2 + n_jobs (a job of odd size leaves a one-pair item)
  const uint32_t items = b.n_sets / 2u + b.n_jobs;
  if (!items || !b.n_sets) return;
  if (b.miller_kv == 9) {
    constexpr uint32_t G = 64 / 27;
    hipLaunchKernelGGL(k_miller_kv<9>, dim3((items + G - 1) / G), dim3(64), 0, st, b, w);
  } else if (b.miller_kv == 6) {
    constexpr uint32_t G = 64 / 18;
    hipLaunchKernelGGL(k_miller_kv<6>, dim3((items + G - 1) / G), dim3(64), 0, st, b, w);
  } else if (b.miller_kv == 2) {
    constexpr uint32_t G = 64 / 6;
    hipLaunchKernelGGL(k_miller_kv<2>, dim3((items + G - 1) / G), dim3(64), 0, st, b, w);
  } else {
    constexpr uint32_t G = 64 / 9;
    hipLaunchKernelGGL(k_miller_kv<3>, dim3((items + G - 1) / G), dim3(64), 0, st, b, w);
  }
}

// the unevaluated lines of every set's H(m) (pairing.h miller_lines), on the
// hash stream right after k_hash: one lane per set
#ifndef BGV_LINES_WAVES
#define BGV_LINES_WAVES 2
#endif
__global__ void __launch_bounds__(64, BGV_LINES_WAVES) k_lines(dev_batch b, dev_work w) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b.n_sets) return;
  miller_lines(w.lines, b.n_sets, i, w.h_aff[i]);
}

void launch_lines(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_sets) hipLaunchKernelGGL(k_lines, dim3((b.n_sets + 63u) / 64u), dim3(64), 0, st, b, w);
}

void launch_miller(hipStream_t st, const dev_batch& b, const dev_work& w) {
  const uint32_t n = b.n_sets / b.pairs_per_item + b.n_jobs;  // >= items (launch_prep)
  if (n) hipLaunchKernelGGL(k_miller, dim3((n + 63u) / 64u), dim3(64), 0, st, b, w, 0u);
}

}  // namespace bgv
