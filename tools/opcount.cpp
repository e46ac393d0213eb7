// Instrumented HOST build of the device arithmetic (lodestar_amd/csrc/*.h)
// that counts Montgomery Fp products per pipeline stage -- the algorithmic
// work W used for the roofline ("frozen by the instrumented
// restatement").  Same code, same formulas as the kernels in
// bgv_kernels.hip, stage by stage.  Prints JSON.
#define BGV_COUNT_OPS 1
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../lodestar_amd/csrc/pairing.h"
namespace bgv { unsigned long long bgv_fpmul_count = 0; }
using namespace bgv;

static int lines_mismatch = 0, lines4_mismatch = 0;
static uint64_t rng = 0x243f6a8885a308d3ull;
static uint64_t rnd64() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

int main(int argc, char** argv) {
  const int k_att = 128, k_sync = 512, per_block = 98;
  // inputs: a valid signature = H(m') compressed, H(m) of a message, table points = multiples of G1
  uint8_t m[32], m2[32];
  for (int i = 0; i < 32; i++) { m[i] = (uint8_t)(i * 7 + 1); m2[i] = (uint8_t)(i * 3 + 5); }
  g2j hs; hash_to_g2(hs, m2);
  g2a hsa; jac_to_aff(hsa, hs);
  uint8_t sig[96];
  { fp_t t; fp_from_mont(t, hsa.x.c1); fp_to_be48(sig, t); fp_from_mont(t, hsa.x.c0); fp_to_be48(sig + 48, t);
    sig[0] |= 0x80 | (fp2_lex_largest(hsa.y) ? 0x20 : 0); }
  g1a pts[64];
  { g1j g, acc; g.x = G1_X_MONT; g.y = G1_Y_MONT; fe_one(g.z); acc = g;
    for (int i = 0; i < 64; i++) { jac_dbl(acc, acc); jac_add(acc, acc, g); jac_to_aff(pts[i], acc); } }

  const int reps = 64;
  double sig_c = 0, sig_dec_c = 0, hash_c = 0, pk_add_c = 0, pk_fix_c = 0, sig_scale_c = 0, miller_c = 0, miller2_c = 0, lines_c = 0, loopl2_c = 0, loopl4_c = 0, fmul_c = 0, g2add_c = 0, aff2_c = 0, fe_c = 0;
  for (int r = 0; r < reps; r++) {
    uint64_t sc = rnd64() | (1ull << 63);  // full 64-bit random scalar (top bit set: worst case)
    sc = rnd64(); if (!sc) sc = 1;
    bgv_fpmul_count = 0;
    g2a a; bool inf; g2_decompress(a, inf, sig);
    sig_dec_c += bgv_fpmul_count;
    g2j j; jac_from_aff(j, a); (void)g2_in_subgroup(j);
    sig_c += bgv_fpmul_count;
    bgv_fpmul_count = 0;
    g2j h; hash_to_g2(h, m); g2a ha; jac_to_aff(ha, h);
    hash_c += bgv_fpmul_count;
    // pk: one mixed add per additional pubkey
    g1j acc; jac_from_aff(acc, pts[0]);
    bgv_fpmul_count = 0;
    for (int i = 1; i < 64; i++) jac_add_aff(acc, acc, pts[i]);
    pk_add_c += (double)bgv_fpmul_count / 63.0;
    bgv_fpmul_count = 0;
    g1j rp; jac_mul_u64_w4(rp, acc, sc); g1a rpa; jac_to_aff(rpa, rp);
    pk_fix_c += bgv_fpmul_count;
    bgv_fpmul_count = 0;
    g2j s2; jac_from_aff(s2, a); g2j rs; jac_mul_u64_w4(rs, s2, sc);
    sig_scale_c += bgv_fpmul_count;
    bgv_fpmul_count = 0;
    g2j t2 = rs; jac_add(t2, t2, rs); jac_add(t2, t2, s2);
    g2add_c += bgv_fpmul_count / 2.0;
    bgv_fpmul_count = 0;
    g2a t2a; jac_to_aff(t2a, t2);
    aff2_c += bgv_fpmul_count;
    bgv_fpmul_count = 0;
    fp12_t f; miller_loop(f, rpa, false, ha, false);
    miller_c += bgv_fpmul_count;
    bgv_fpmul_count = 0;
    fp12_t f2; miller_loop2(f2, rpa, ha, rpa, ha);  // C4 (n >= 65536): two sets per work item
    miller2_c += bgv_fpmul_count;
    // fixed-argument lines (BGV_LINES, C4): lines of H(m) on the hash stream, then the loop over them
    static fp2_t lines[3 * MILLER_STEPS];
    bgv_fpmul_count = 0;
    miller_lines(lines, 1, 0, ha);
    lines_c += bgv_fpmul_count;
    bgv_fpmul_count = 0;
    fp12_t f3; miller_loop_lines(f3, lines, 1, rpa, 0, rpa, 0, true);
    loopl2_c += bgv_fpmul_count;
    if (memcmp(&f3, &f2, sizeof f2) != 0) lines_mismatch++;
    // four pairs per item (pairs_per_item = 4): four sets' lines at stride 4;
    // f4 equals the product of the two two-pair values exactly, and an item
    // with cnt < 4 live pairs equals the product over its live pairs
    {
      static fp2_t l4[3 * MILLER_STEPS * 4];
      g2a q4[4] = {ha, hsa, ha, hsa};
      for (int i = 0; i < 4; i++) miller_lines(l4, 4, i, q4[i]);
      const g1a* P = &pts[(r * 4) % 60];
      bgv_fpmul_count = 0;
      fp12_t f4; miller_loop_lines4(f4, l4, 4, P[0], P[1], P[2], P[3], 0, 1, 2, 3, 4);
      loopl4_c += bgv_fpmul_count;
      fp12_t fa, fb, fab;
      miller_loop_lines(fa, l4, 4, P[0], 0, P[1], 1, true);
      miller_loop_lines(fb, l4, 4, P[2], 2, P[3], 3, true);
      fp12_mul(fab, fa, fb);
      if (memcmp(&f4, &fab, sizeof f4) != 0) lines4_mismatch++;
      fp12_t f4c3, fc, fac;
      miller_loop_lines4(f4c3, l4, 4, P[0], P[1], P[2], P[0], 0, 1, 2, 0, 3);  // dead fourth pair
      miller_loop_lines(fc, l4, 4, P[2], 2, P[2], 2, false);
      fp12_mul(fac, fa, fc);
      if (memcmp(&f4c3, &fac, sizeof f4) != 0) lines4_mismatch++;
      fp12_t f4c1, fd;
      miller_loop_lines4(f4c1, l4, 4, P[1], P[1], P[1], P[1], 1, 1, 1, 1, 1);
      miller_loop_lines(fd, l4, 4, P[1], 1, P[1], 1, false);
      if (memcmp(&f4c1, &fd, sizeof f4) != 0) lines4_mismatch++;
    }
    bgv_fpmul_count = 0;
    fp12_t g; fp12_mul(g, f, f);
    fmul_c += bgv_fpmul_count;
    if (r == 0) { bgv_fpmul_count = 0; fp12_t e; fp12_final_exp(e, f); fe_c = bgv_fpmul_count; }
  }
  // per-job bucket MSM of the signatures (bgv_kernels.hip k_msm_*), one 98-set job
  double msm_c = 0, msm_bucket_c = 0;
  {
    g2a pts[per_block];
    g2j acc; jac_from_aff(acc, hsa);
    for (int i = 0; i < per_block; i++) { jac_dbl(acc, acc); jac_to_aff(pts[i], acc); }
    uint64_t sc[per_block];
    for (int i = 0; i < per_block; i++) { sc[i] = rnd64(); if (!sc[i]) sc[i] = 1; }
    bgv_fpmul_count = 0;
    g2j win[16];
    g2j bks[16][15]; uint32_t masks[16];
    for (int w = 0; w < 16; w++) {  // k_msm_bucket (ST_SIG_SCALE)
      g2j* bk = bks[w]; uint32_t mask = 0;
      for (int i = 0; i < per_block; i++) {
        const uint32_t d = (uint32_t)(sc[i] >> (4 * w)) & 15u;
        if (!d) continue;
        if ((mask >> d) & 1u) jac_add_aff(bk[d - 1], bk[d - 1], pts[i]);
        else { jac_from_aff(bk[d - 1], pts[i]); mask |= 1u << d; }
      }
      masks[w] = mask;
    }
    msm_bucket_c = (double)bgv_fpmul_count / per_block;
    for (int w = 0; w < 16; w++) {  // k_msm_window + k_msm_job (ST_S_TREE)
      g2j* bk = bks[w]; const uint32_t mask = masks[w];
      g2j run, tot; jac_set_inf(run); jac_set_inf(tot);
      for (int d = 15; d >= 1; d--) { if ((mask >> d) & 1u) jac_add(run, run, bk[d - 1]); jac_add(tot, tot, run); }
      win[w] = tot;
    }
    g2j s = win[15];
    for (int w = 14; w >= 0; w--) { for (int k = 0; k < 4; k++) jac_dbl(s, s); jac_add(s, s, win[w]); }
    g2a sa; jac_to_aff(sa, s);
    msm_c = (double)bgv_fpmul_count / per_block;
  }
  sig_c /= reps; sig_dec_c /= reps; hash_c /= reps; pk_add_c /= reps; pk_fix_c /= reps; sig_scale_c /= reps; miller_c /= reps; miller2_c /= reps; lines_c /= reps; loopl2_c /= reps; loopl4_c /= reps;
  fmul_c /= reps; g2add_c /= reps; aff2_c /= reps;
  // C4 block mix: 95 sets of k=128, 1 of k=512, 2 singles -> mean pubkeys per set
  const double mean_k = (95.0 * k_att + k_sync + 2.0) / per_block;
  const double pk_c = (mean_k - 1.0) * pk_add_c + pk_fix_c;
  // trees per set (C4: 98 sets per job, 1024 jobs)
  const double s_tree_per_set_path = g2add_c * (per_block - 1.0) / per_block + aff2_c / per_block;
  (void)s_tree_per_set_path;  // the per-set path (small batches): sig_scale = g2_mul_u64, then this tree
  // C4 (>= 65,536 sets): the MSM buckets are sig_scale; window sums, Horner and affine are the s-tree stage
  const double s_tree = msm_c - msm_bucket_c;
  const double pk_gather = (mean_k - 1.0) * pk_add_c;
  const double f_tree = fmul_c * (per_block) / per_block;  // (98-1) set products + the job pair, per set
  // Miller stage at C4: 49 two-set items (shared f squaring, pairing.h miller_loop2) + the job pair
  const double miller_set = miller2_c / 2.0;           // ST_MILLER: the set pairs
  const double miller_jobs = miller_c / per_block;      // ST_MILLER_JOBS: one (-G1, S_job) pair per job
  printf("{\n \"generator\": \"tools/opcount.cpp (instrumented host build of lodestar_amd/csrc)\",\n");
  printf(" \"unit\": \"Montgomery Fp products (fp_mul calls, squares included) per signature set\",\n");
  printf(" \"workload\": \"C4 block mix: 95 x k=128, 1 x k=512, 2 x k=1 per 98-set job; random 64-bit scalars\",\n");
  printf(" \"mean_pubkeys_per_set\": %.3f,\n", mean_k);
  printf(" \"components\": {\"g2_decompress_subgroup\": %.1f, \"hash_to_g2_affine\": %.1f, \"g1_mixed_add\": %.2f, "
         "\"g1_mul_u64_affine\": %.1f, \"g2_mul_u64\": %.1f, \"g2_add\": %.1f, \"g2_to_affine\": %.1f, \"miller_loop_pair\": %.1f, "
         "\"miller_loop_2pairs\": %.1f, \"fp12_mul\": %.1f, \"final_exp\": %.1f, \"sig_msm_per_set\": %.1f},\n",
         sig_c, hash_c, pk_add_c, pk_fix_c, sig_scale_c, g2add_c, aff2_c, miller_c, miller2_c, fmul_c, fe_c, msm_c);
  printf(" \"per_set\": {\"sig_decode_subgroup\": %.1f, \"hash_to_g2\": %.1f, \"pk_gather\": %.1f, \"pk_aggregate_scale\": %.1f, "
         "\"sig_scale\": %.1f, \"sig_sum_tree\": %.1f, \"miller_loop\": %.1f, \"miller_loop_jobs\": %.1f, \"miller_product_tree\": %.1f},\n",
         sig_c, hash_c, pk_gather, pk_fix_c, msm_bucket_c, s_tree, miller_set, miller_jobs, f_tree);
  // fixed-argument lines at C4: the lines are their own (untimed) step, the
  // Miller stage loops over them; the two-pair value is bit-identical
  printf(" \"g2_decompress_only\": %.1f,\n", sig_dec_c);
  printf(" \"per_set_lines\": {\"miller_lines\": %.1f, \"miller_loop\": %.1f, \"loop_values_match\": %s},\n",
         lines_c, loopl2_c / 2.0, lines_mismatch ? "false" : "true");
  // four pairs per item (C4 blocks of 98 sets: 24 items of 4 and one of 2,
  // whose dead pairs still cost a full item): per set = loop4 x 25 / 98
  printf(" \"per_set_lines4\": {\"miller_lines\": %.1f, \"miller_loop\": %.1f, \"miller_loop_full_items\": %.1f, "
         "\"miller_product_tree\": %.1f, \"loop_values_match\": %s},\n",
         lines_c, loopl4_c * 25.0 / per_block, loopl4_c / 4.0, fmul_c * 25.0 / per_block, lines4_mismatch ? "false" : "true");
  printf(" \"per_set_total\": %.1f,\n", sig_c + hash_c + pk_c + msm_c + miller_set + miller_jobs + f_tree);
  printf(" \"per_set_total_lines\": %.1f,\n", sig_c + hash_c + pk_c + msm_c + lines_c + loopl2_c / 2.0 + miller_jobs + f_tree);
  printf(" \"per_set_total_lines4\": %.1f\n}\n", sig_c + hash_c + pk_c + msm_c + lines_c + loopl4_c * 25.0 / per_block + miller_jobs +
         fmul_c * 25.0 / per_block);
  return 0;
}
