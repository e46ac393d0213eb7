// Latency-mode kernels with cooperative G2 arithmetic (coop_g2.h): the
// subgroup check / [r_i] sigma_i pair and the cofactor clearing of
// hash_to_G2 for batches below 65,536 sets, nine lanes per point.  Their own
// translation unit: they run at 1 wave/SIMD (launch bounds 64, 1), and the
// non-inlined curve helpers they share with k_sig would otherwise be
// compiled for their register budget (k_sig went to 321 VGPRs).
#ifndef BGV_FPMUL_CALL
#define BGV_FPMUL_CALL 1
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
#include "bgv_internal.h"
#include "coop_g2.h"
#include "kv_g2.h"
#include "coop_g1.h"

#ifndef BGV_KV_CLEAR
#define BGV_KV_CLEAR 1  // three-lane clearing in views (kv_g2.h)
#endif
#ifndef BGV_KV9
#define BGV_KV9 1  // nine-lane G2 kernels in views (kv_g2.h)
#endif
#ifndef BGV_KV9_LEVEL
#define BGV_KV9_LEVEL 0
#endif

namespace bgv {

// Latency mode with cooperative G2 arithmetic (coop_g2.h, BGV_COOP_G2):
// nine lanes per point, seven points per wave.  Lane 63 and groups past
// n_sets run on a copy of set 0 into their own scratch and write nothing.
__global__ void __launch_bounds__(64, 1) k_sig_split_coop(dev_batch b, dev_work w) {
  __shared__ cg_scratch sm[CG_GROUPS + 1];
  __shared__ g2j tabs[CG_GROUPS + 1][16];
  const uint32_t nbg = (b.n_sets + CG_GROUPS - 1) / CG_GROUPS;
  const bool check = blockIdx.x < nbg;
  const uint32_t lane = threadIdx.x, grp = lane / CG_LANES, r9 = lane % CG_LANES, s = r9 / 3, q = r9 % 3;
  const uint32_t i0 = (check ? blockIdx.x : blockIdx.x - nbg) * CG_GROUPS + grp;
  const bool own = grp < CG_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  const bool lead = own && s == 0 && q == 0;
  const bool live = w.sig_code[i] == C_OK && !w.sig_inf[i];  // decode outcome (k_sig_dec)
  g2j p;
  jac_from_aff(p, w.sig_aff[i]);
  if (check) {
    const bool ok = !live || cg_in_subgroup<3>(&sm[grp], s, q, p);
    if (lead) w.sig_grp[i] = ok ? 1u : 0u;
  } else {
    g2j r;
    if (live) cg_mul_u64_w4<3>(&sm[grp], tabs[grp], s, q, r, p, b.scalars[i]);
    else jac_set_inf(r);  // infinity signature: blst skips it (adds the identity)
    if (lead) w.rsig[i] = r;
  }
}

__global__ void __launch_bounds__(64, 1) k_hash_clear_coop(dev_batch b, dev_work w) {
  __shared__ cg_scratch sm[CG_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / CG_LANES, r9 = lane % CG_LANES, s = r9 / 3, q = r9 % 3;
  const uint32_t i0 = blockIdx.x * CG_GROUPS + grp;
  const bool own = grp < CG_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  g2j r, h;
  cg_add<3>(&sm[grp], s, q, r, w.q_part[2u * i], w.q_part[2u * i + 1u]);
  cg_clear_cofactor<3>(&sm[grp], s, q, h, r);
  if (own && s == 0 && q == 0) {
    g2a ha;
    jac_to_aff(ha, h);
    w.h_aff[i] = ha;
  }
}

// The cofactor clearing on THREE lanes per point (coop_g2.h with one slot:
// the sub-lanes of one Fp2 product, products in turn), 21 points per wave:
// half the SIMD-time of the nine-lane layout for mid-size batches, where
// nine lanes per point oversubscribe the chip (12,544 sets: 1,792 waves)
constexpr int CG3_GROUPS = 21;
__global__ void __launch_bounds__(64, 1) k_hash_clear_trio(dev_batch b, dev_work w) {
  __shared__ cg_scratch sm[CG3_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / 3u, q = lane % 3u;
  const uint32_t i0 = blockIdx.x * CG3_GROUPS + grp;
  const bool own = grp < (uint32_t)CG3_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  g2j r, h;
  cg_add<1>(&sm[grp], 0u, q, r, w.q_part[2u * i], w.q_part[2u * i + 1u]);
  cg_clear_cofactor<1>(&sm[grp], 0u, q, h, r);
  if (own && q == 0) {
    g2a ha;
    jac_to_aff(ha, h);
    w.h_aff[i] = ha;
  }
}

// The same clearing in Karatsuba views (kv_g2.h): each lane of the three
// holds one Fp view of every Fp2 value, so the point formulas' additions are
// one Fp operation per lane and no operand is selected before a product
constexpr int KV1_GROUPS = 21;
__global__ void __launch_bounds__(64, 1) k_hash_clear_kv(dev_batch b, dev_work w) {
  __shared__ kv_scratch<1> sm[KV1_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / 3u, q = lane % 3u;
  const uint32_t i0 = blockIdx.x * KV1_GROUPS + grp;
  const bool own = grp < (uint32_t)KV1_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  const kv_grp<1> g{&sm[grp], grp, 0u, q};
  kv_init<1>(g.sc, 0u, q);
  kv_pt p0, p1, r, h;
  kv_load(p0, w.q_part[2u * i], q);
  kv_load(p1, w.q_part[2u * i + 1u], q);
  kv_add<1>(g, r, p0, p1);
  kv_clear_cofactor<1>(g, h, r);
  g2j hj;
  kv_gather<1>(g, hj, h);
  if (own && q == 0) {
    g2a ha;
    jac_to_aff(ha, hj);
    w.h_aff[i] = ha;
  }
}

// nine lanes per point in views (three slots x three views): the layouts of
// k_hash_clear_coop / k_sig_split_coop / k_s_level_coop / k_msm_job_coop
// with kv_g2.h arithmetic
constexpr int KV3_GROUPS = 7;
__global__ void __launch_bounds__(64, 1) k_hash_clear_kv9(dev_batch b, dev_work w) {
  __shared__ kv_scratch<3> sm[KV3_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / 9u, r9 = lane % 9u, s = r9 / 3u, q = r9 % 3u;
  const uint32_t i0 = blockIdx.x * KV3_GROUPS + grp;
  const bool own = grp < (uint32_t)KV3_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  const kv_grp<3> g{&sm[grp], grp, s, q};
  kv_init<3>(g.sc, s, q);
  kv_pt p0, p1, r, h;
  kv_load(p0, w.q_part[2u * i], q);
  kv_load(p1, w.q_part[2u * i + 1u], q);
  kv_add<3>(g, r, p0, p1);
  kv_clear_cofactor<3>(g, h, r);
  g2j hj;
  kv_gather<3>(g, hj, h);
  if (own && s == 0 && q == 0) {
    g2a ha;
    jac_to_aff(ha, hj);
    w.h_aff[i] = ha;
  }
}

__global__ void __launch_bounds__(64, 1) k_sig_split_kv9(dev_batch b, dev_work w) {
  __shared__ kv_scratch<3> sm[KV3_GROUPS + 1];
  __shared__ g2j tabs[KV3_GROUPS][16];
  const uint32_t nbg = (b.n_sets + KV3_GROUPS - 1) / KV3_GROUPS;
  const bool check = blockIdx.x < nbg;
  const uint32_t lane = threadIdx.x, grp = lane / 9u, r9 = lane % 9u, s = r9 / 3u, q = r9 % 3u;
  const uint32_t i0 = (check ? blockIdx.x : blockIdx.x - nbg) * KV3_GROUPS + grp;
  const bool own = grp < (uint32_t)KV3_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  const bool lead = own && s == 0 && q == 0;
  const bool live = w.sig_code[i] == C_OK && !w.sig_inf[i];  // decode outcome (k_sig_dec)
  const kv_grp<3> g{&sm[grp], grp, s, q};
  kv_init<3>(g.sc, s, q);
  g2j pj;
  jac_from_aff(pj, w.sig_aff[i]);
  kv_pt p;
  kv_load(p, pj, q);
  if (check) {
    const bool ok = kv_in_subgroup<3>(g, p);
    if (lead) w.sig_grp[i] = (!live || ok) ? 1u : 0u;
  } else {
    kv_pt r;
    // lane 63 (grp 7) computes on group 6's table without writing it
    kv_mul_u64_w4<3>(g, tabs[grp < (uint32_t)KV3_GROUPS ? grp : KV3_GROUPS - 1u], grp < (uint32_t)KV3_GROUPS, r, p, b.scalars[i]);
    g2j rj;
    kv_gather<3>(g, rj, r);
    if (!live) jac_set_inf(rj);  // infinity signature: blst skips it (adds the identity)
    if (lead) w.rsig[i] = rj;
  }
}

// k_pk (bgv_kernels.hip) on three lanes per set (coop_g1.h): the chunk sums
// folded per set, then [r_i] PK_i and the affine conversion.  The latency
// mode's path to the Miller loop waits for it (3,136 sets: one-lane k_pk
// 1.6 ms after the gather, while the hash chain ends ~0.6 ms earlier).
constexpr int G1C_GROUPS = 21;
__global__ void __launch_bounds__(64, 1) k_pk_coop(dev_batch b, dev_work w) {
  __shared__ g1c_scratch sm[G1C_GROUPS + 1];
  __shared__ g1j tabs[G1C_GROUPS][16];
  const uint32_t lane = threadIdx.x, grp = lane / 3u, s = lane % 3u;
  const uint32_t i0 = blockIdx.x * G1C_GROUPS + grp;
  const bool own = grp < (uint32_t)G1C_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  const g1c_grp g{&sm[grp], s};
  g1j acc;
  jac_set_inf(acc);
  const uint32_t c0 = w.chunk_off[i], c1 = w.chunk_off[i + 1];
  bool range_err = c1 > b.chunk_bound || b.pk_off[i + 1] < b.pk_off[i];
  const uint32_t cend = range_err ? c0 : c1;
  // the wave walks its longest chunk list together (rounds stay wave-wide)
  uint32_t nmax = cend - c0;
  for (uint32_t off = 32; off >= 1; off >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, off, 64));
  for (uint32_t k = 0; k < nmax; k++) {
    const bool live = c0 + k < cend;
    g1j pp;
    if (live) pp = w.pk_part[c0 + k];
    else jac_set_inf(pp);
    if (live && !jac_is_inf(pp) && fp_is_zero(pp.x)) range_err = true;
    g1c_add(g, acc, acc, pp);
  }
  int32_t code = C_OK;
  if (range_err) code = C_INDEX_RANGE;
  else if (jac_is_inf(acc)) code = C_PK_IS_INFINITY;
  g1a out;
  if (w.pk_agg && own && s == 0) {  // bgv_debug_stages: the aggregate before scaling
    if (code != C_OK || !jac_to_aff(out, acc)) { fp_set_zero(out.x); fp_set_zero(out.y); }
    w.pk_agg[i] = out;
  }
  g1j rp;
  g1c_mul_u64_w4(g, tabs[grp < (uint32_t)G1C_GROUPS ? grp : G1C_GROUPS - 1u], grp < (uint32_t)G1C_GROUPS, rp, acc,
                 b.scalars[i]);
  if (!own || s != 0) return;
  if (code == C_OK) {
    jac_to_aff(out, rp);
  } else {
    fp_set_zero(out.x);
    fp_set_zero(out.y);
  }
  w.rpk_aff[i] = out;
  w.pk_code[i] = code;
}

void launch_pk_coop(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_sets) hipLaunchKernelGGL(k_pk_coop, dim3((b.n_sets + G1C_GROUPS - 1) / G1C_GROUPS), dim3(64), 0, st, b, w);
}

void launch_hash_clear_trio(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (!b.n_sets) return;
  if (BGV_KV_CLEAR)
    hipLaunchKernelGGL(k_hash_clear_kv, dim3((b.n_sets + KV1_GROUPS - 1) / KV1_GROUPS), dim3(64), 0, st, b, w);
  else
    hipLaunchKernelGGL(k_hash_clear_trio, dim3((b.n_sets + CG3_GROUPS - 1) / CG3_GROUPS), dim3(64), 0, st, b, w);
}

// One level of the per-job signature sum (bgv_kernels.hip k_s_level) on nine
// lanes per addition (coop_g2.h cg_add, 6 rounds of one Fp product):
// rsig[i] += rsig[i + s] for every set i an even multiple of s past its job's
// start.  A one-lane G2 addition costs ~140 us of latency (k_s_level: 0.15 ms
// per level at 3,136 sets); waves without a live addition leave at once.
__global__ void __launch_bounds__(64, 1) k_s_level_coop(dev_batch b, dev_work w, uint32_t s) {
  __shared__ cg_scratch sm[CG_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / CG_LANES, r9 = lane % CG_LANES, sl = r9 / 3, q = r9 % 3;
  const uint32_t i0 = blockIdx.x * CG_GROUPS + grp;
  bool own = grp < CG_GROUPS && i0 < b.n_sets;
  if (own) {
    const uint32_t j = w.set_job[i0];
    own = ((i0 - b.job_off[j]) % (2u * s)) == 0 && i0 + s < b.job_off[j + 1];
  }
  if (!__any(own)) return;  // wave-uniform
  const uint32_t i = own ? i0 : 0u, k = own ? i0 + s : 0u;
  g2j r;
  cg_add<3>(&sm[grp], sl, q, r, w.rsig[i], w.rsig[k]);
  if (own && sl == 0 && q == 0) w.rsig[i] = r;
}

__global__ void __launch_bounds__(64, 1) k_s_level_kv9(dev_batch b, dev_work w, uint32_t s) {
  __shared__ kv_scratch<3> sm[KV3_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / 9u, r9 = lane % 9u, sl = r9 / 3u, q = r9 % 3u;
  const uint32_t i0 = blockIdx.x * KV3_GROUPS + grp;
  bool own = grp < (uint32_t)KV3_GROUPS && i0 < b.n_sets;
  if (own) {
    const uint32_t j = w.set_job[i0];
    own = ((i0 - b.job_off[j]) % (2u * s)) == 0 && i0 + s < b.job_off[j + 1];
  }
  if (!__any(own)) return;  // wave-uniform
  const uint32_t i = own ? i0 : 0u, k = own ? i0 + s : 0u;
  const kv_grp<3> g{&sm[grp], grp, sl, q};
  kv_init<3>(g.sc, sl, q);
  kv_pt a, c, r;
  kv_load(a, w.rsig[i], q);
  kv_load(c, w.rsig[k], q);
  kv_add<3>(g, r, a, c);
  g2j rj;
  kv_gather<3>(g, rj, r);
  if (own && sl == 0 && q == 0) w.rsig[i] = rj;
}

// per job: S_job = sum_w 16^w S_w from the MSM's 16 window sums (msm_win,
// k_msm_digit / k_msm_window) by Horner on nine lanes per job (seven jobs per
// wave): 60 cooperative doublings (3 rounds of one Fp product each) and 15
// additions, against the one-lane form's 60 doublings of ~16 sequential Fp
// products each (bgv_kernels.hip k_msm_job: 2.8 ms at 12,544 sets).  Codes as
// k_job_s (first failing set code, signatures before pubkeys).  S_job's affine
// value does not depend on the order of the additions.
__global__ void __launch_bounds__(64, 1) k_msm_job_coop(dev_batch b, dev_work w) {
  #if BGV_KV9
  __shared__ kv_scratch<3> smk[KV3_GROUPS + 1];
#else
  __shared__ cg_scratch sm[CG_GROUPS + 1];
#endif
  const uint32_t lane = threadIdx.x, grp = lane / CG_LANES, r9 = lane % CG_LANES, sl = r9 / 3, q = r9 % 3;
  const uint32_t j0 = blockIdx.x * CG_GROUPS + grp;
  const bool own = grp < CG_GROUPS && j0 < b.n_jobs;
  const uint32_t j = own ? j0 : 0u;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  int32_t code = C_OK;
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.sig_code[i];
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.pk_code[i];
  if (end == beg) code = C_EMPTY_JOB;
  const g2j* win = w.msm_win + 16u * j;
  g2j s;
#if BGV_KV9
  {
    const kv_grp<3> g{&smk[grp], grp, sl, q};
    kv_init<3>(g.sc, sl, q);
    kv_pt acc, e;
    kv_load(acc, win[15], q);
#pragma unroll 1
    for (int k = 14; k >= 0; k--) {
      kv_dbl<3>(g, acc, acc);
      kv_dbl<3>(g, acc, acc);
      kv_dbl<3>(g, acc, acc);
      kv_dbl<3>(g, acc, acc);
      kv_load(e, win[k], q);
      kv_add<3>(g, acc, acc, e);
    }
    kv_gather<3>(g, s, acc);
  }
#else
  s = win[15];
#pragma unroll 1
  for (int k = 14; k >= 0; k--) {
    cg_dbl<3>(&sm[grp], sl, q, s, s);
    cg_dbl<3>(&sm[grp], sl, q, s, s);
    cg_dbl<3>(&sm[grp], sl, q, s, s);
    cg_dbl<3>(&sm[grp], sl, q, s, s);
    cg_add<3>(&sm[grp], sl, q, s, s, win[k]);
  }
#endif
  if (!own || sl != 0 || q != 0) return;
  g2a sa;
  sa.x = fp2_zero();
  sa.y = fp2_zero();
  uint32_t inf = 1;
  if (code == C_OK) inf = jac_to_aff(sa, s) ? 0u : 1u;
  w.s_aff[j] = sa;
  w.s_inf[j] = inf;
  w.job_code[j] = code;
}

void launch_msm_job_coop(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_jobs) hipLaunchKernelGGL(k_msm_job_coop, dim3((b.n_jobs + CG_GROUPS - 1) / CG_GROUPS), dim3(64), 0, st, b, w);
}

void launch_s_level_coop(hipStream_t st, const dev_batch& b, const dev_work& w, uint32_t s) {
  if (!b.n_sets) return;
  // the one-addition levels stay on coop_g2.h: the view form's load and
  // gather of a lone addition cost more than it saves (3,136 sets: 0.045
  // against 0.027 ms per level)
  if (BGV_KV9 && BGV_KV9_LEVEL) hipLaunchKernelGGL(k_s_level_kv9, dim3((b.n_sets + KV3_GROUPS - 1) / KV3_GROUPS), dim3(64), 0, st, b, w, s);
  else hipLaunchKernelGGL(k_s_level_coop, dim3((b.n_sets + CG_GROUPS - 1) / CG_GROUPS), dim3(64), 0, st, b, w, s);
}

void launch_sig_split_coop(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (!b.n_sets) return;
  if (BGV_KV9)
    hipLaunchKernelGGL(k_sig_split_kv9, dim3(2u * ((b.n_sets + KV3_GROUPS - 1) / KV3_GROUPS)), dim3(64), 0, st, b, w);
  else
    hipLaunchKernelGGL(k_sig_split_coop, dim3(2u * ((b.n_sets + CG_GROUPS - 1) / CG_GROUPS)), dim3(64), 0, st, b, w);
}

void launch_hash_clear_coop(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (!b.n_sets) return;
  if (BGV_KV9) hipLaunchKernelGGL(k_hash_clear_kv9, dim3((b.n_sets + KV3_GROUPS - 1) / KV3_GROUPS), dim3(64), 0, st, b, w);
  else hipLaunchKernelGGL(k_hash_clear_coop, dim3((b.n_sets + CG_GROUPS - 1) / CG_GROUPS), dim3(64), 0, st, b, w);
}

}  // namespace bgv
