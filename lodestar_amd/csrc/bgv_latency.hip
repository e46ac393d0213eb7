// Latency-mode kernels with cooperative G2 arithmetic (coop_g2_fd.h): the
// subgroup check / [r_i] sigma_i pair and the cofactor clearing of
// hash_to_G2 for small batches, twelve lanes per point over the signed-digit
// field (fd.h).  Their own
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
#include "coop_g2_fd.h"

namespace bgv {

// Latency mode with cooperative G2 arithmetic (coop_g2_fd.h): twelve lanes
// per point, five points per wave.  Lanes 60..63 and groups past n_sets run
// on a copy of set 0 into their own scratch and write nothing.  Inputs are
// converted into the signed-digit field by a product round with 2^400, the
// results back by one with 2^384 (canonical, fp.h form).
__global__ void __launch_bounds__(64, 1) k_sig_split_coop(dev_batch b, dev_work w) {
  __shared__ gd_scratch sm[GD_GROUPS + 1];
  __shared__ gd2j tabs[GD_GROUPS + 1][16];
  const uint32_t nbg = (b.n_sets + GD_GROUPS - 1) / GD_GROUPS;
  const bool check = blockIdx.x < nbg;
  const uint32_t lane = threadIdx.x, grp = lane / GD_LANES, r12 = lane % GD_LANES, s = r12 / 4, q = r12 % 4;
  const uint32_t i0 = (check ? blockIdx.x : blockIdx.x - nbg) * GD_GROUPS + grp;
  const bool own = grp < GD_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  const bool lead = own && s == 0 && q == 0;
  const bool live = w.sig_code[i] == C_OK && !w.sig_inf[i];  // decode outcome (k_sig_dec)
  gd_dev rp{&sm[grp], s, q};
  gd2j p;
  gd_from_g2a(rp, p, w.sig_aff[i]);
  if (check) {
    const bool ok = !live || gd_in_subgroup(rp, p);
    if (lead) w.sig_grp[i] = ok ? 1u : 0u;
  } else {
    g2j r;
    if (live) {
      gd2j rd;
      gd_mul_u64_w4(rp, tabs[grp], s == 0 && q == 0, rd, p, b.scalars[i]);
      gd_to_g2j(rp, r, rd);
    } else {
      jac_set_inf(r);  // infinity signature: blst skips it (adds the identity)
    }
    if (lead) w.rsig[i] = r;
  }
}

__global__ void __launch_bounds__(64, 1) k_hash_clear_coop(dev_batch b, dev_work w) {
  __shared__ gd_scratch sm[GD_GROUPS + 1];
  const uint32_t lane = threadIdx.x, grp = lane / GD_LANES, r12 = lane % GD_LANES, s = r12 / 4, q = r12 % 4;
  const uint32_t i0 = blockIdx.x * GD_GROUPS + grp;
  const bool own = grp < GD_GROUPS && i0 < b.n_sets;
  const uint32_t i = own ? i0 : 0u;
  gd_dev rp{&sm[grp], s, q};
  gd2j q0, q1, r, h;
  gd_from_g2j(rp, q0, w.q_part[2u * i]);
  gd_from_g2j(rp, q1, w.q_part[2u * i + 1u]);
  gd_add(rp, r, q0, q1);
  gd_clear_cofactor(rp, h, r);
  g2j hj;
  gd_to_g2j(rp, hj, h);
  if (own && s == 0 && q == 0) {
    g2a ha;
    jac_to_aff(ha, hj);
    w.h_aff[i] = ha;
  }
}

void launch_sig_split_coop(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_sets) hipLaunchKernelGGL(k_sig_split_coop, dim3(2u * ((b.n_sets + GD_GROUPS - 1) / GD_GROUPS)), dim3(64), 0, st, b, w);
}

void launch_hash_clear_coop(hipStream_t st, const dev_batch& b, const dev_work& w) {
  if (b.n_sets) hipLaunchKernelGGL(k_hash_clear_coop, dim3((b.n_sets + GD_GROUPS - 1) / GD_GROUPS), dim3(64), 0, st, b, w);
}

}  // namespace bgv
