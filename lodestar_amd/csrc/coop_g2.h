// Cooperative G2 point arithmetic for the latency mode (small batches):
// NINE lanes per point.  Every lane of a group holds the whole point and
// runs the additions redundantly; only the Fp2 products are distributed:
// a round computes up to three Fp2 products, lane (s, q) (s = slot 0..2,
// q = Karatsuba sub-product 0..2) one Fp product each, exchanged through
// LDS inside one wave.  A point doubling is 3 rounds, an addition 6, so a
// 64-bit scalar multiplication costs ~370 rounds of ONE Fp product of
// latency instead of ~2,100 sequential Fp products on one lane.
//
// Formulas and their order are those of curve.h (dbl-2009-l, add-2007-bl
// with the exceptional cases, the 4-bit fixed window of jac_mul_u64_w4, the
// x-chain of jac_mul_abs_x, Budroni-Pintore h_eff), so the Jacobian
// coordinates equal the one-lane kernels' (GPU test: latency mode on/off).
#pragma once
#include "miller_coop.h"
#include "lds.h"

namespace bgv {

constexpr int CG_LANES = 9;
constexpr int CG_GROUPS = 64 / CG_LANES;  // 7 points per wave

#ifndef BGV_CG_SPLIT_COMBINE
#define BGV_CG_SPLIT_COMBINE 1
#endif
#ifndef BGV_CG_TRIO_BATCH
#define BGV_CG_TRIO_BATCH 1
#endif

// force-inline the round and the point steps into the latency kernels (A/B knob)
#ifndef BGV_CG_INLINE
#define BGV_CG_INLINE 1  // k_hash_clear_coop 1.86 -> 1.77 ms, k_sig_split_coop 1.24 -> 1.17 ms (scratch 1936 -> 1504 B/lane)
#endif
#if BGV_CG_INLINE
#define BGV_CGF __device__ __forceinline__
#else
#define BGV_CGF __device__
#endif

struct cg_scratch {
  fp_t P[3][3];  // [slot][sub-product]
  fp_t O[3][2];  // [slot][c0, c1] (BGV_CG_SPLIT_COMBINE)
};

__device__ __forceinline__ fp2_t cg_sel(uint32_t s, const fp2_t& x0, const fp2_t& x1, const fp2_t& x2) {
  return s == 0 ? x0 : (s == 1 ? x1 : x2);
}

__device__ __forceinline__ void cg_combine(fp2_t& o, const fp_t* P) {
  fp_t w;
  fp_add_sub(w, P[0], P[1], o.c0, P[0], P[1]);
  fp_sub(o.c1, P[2], w);
}

// one Fp2 product o = a * b on the three sub-lanes q of a one-slot group
// (SLOTS = 1: three lanes per point): q0 a0 b0, q1 a1 b1, q2 (a0 + a1)(b0 + b1)
BGV_CGF void cg_prod1(cg_scratch* S, uint32_t q, const fp2_t& a, const fp2_t& b, fp2_t& o) {
  fp_t u, v;
  if (q == 0) {
    u = a.c0;
    v = b.c0;
  } else if (q == 1) {
    u = a.c1;
    v = b.c1;
  } else {
    fp_add_lazy(u, a.c0, a.c1);  // < 2p, product inputs only
    fp_add_lazy(v, b.c0, b.c1);
  }
  fp_t r;
  fp_mul(r, u, v);
  BGV_LDS cg_scratch* L = (BGV_LDS cg_scratch*)S;
  lds_put(&L->P[0][q], r);
  coop_wave_sync();
  // every lane combines (one dual add/sub and a subtraction: the same issue
  // cost as two lanes combining, without a second exchange)
  const fp_t p0 = lds_get(&L->P[0][0]), p1 = lds_get(&L->P[0][1]), p2 = lds_get(&L->P[0][2]);
  fp_t w;
  fp_add_sub(w, p0, p1, o.c0, p0, p1);
  fp_sub(o.c1, p2, w);
  coop_wave_sync();
}

// o_k = a_k * b_k for k < n (n <= 3); every lane of the group calls it.
// SLOTS = 3: one round, slot s computes product s; SLOTS = 1: n products in turn
template <int SLOTS>
BGV_CGF void cg_round(cg_scratch* S, uint32_t s, uint32_t q, int n, const fp2_t& a0, const fp2_t& b0,
                         const fp2_t& a1, const fp2_t& b1, const fp2_t& a2, const fp2_t& b2, fp2_t& o0, fp2_t& o1,
                         fp2_t& o2) {
  if constexpr (SLOTS == 1) {
#if BGV_CG_TRIO_BATCH
    // three lanes: lane q forms Karatsuba sub-product q of EVERY Fp2 product
    // of the round (n Fp products in a row), then ONE exchange and every lane
    // combines the n products: n product latencies + 1 exchange, against n x
    // (1 product + 1 exchange) when the products go through one at a time
    BGV_LDS cg_scratch* L = (BGV_LDS cg_scratch*)S;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k >= n) break;
      const fp2_t& a = k == 0 ? a0 : (k == 1 ? a1 : a2);
      const fp2_t& b = k == 0 ? b0 : (k == 1 ? b1 : b2);
      fp_t u, v;
      if (q == 0) {
        u = a.c0;
        v = b.c0;
      } else if (q == 1) {
        u = a.c1;
        v = b.c1;
      } else {
        fp_add_lazy(u, a.c0, a.c1);  // < 2p, product inputs only
        fp_add_lazy(v, b.c0, b.c1);
      }
      fp_t r;
      fp_mul(r, u, v);
      lds_put(&L->P[k][q], r);
    }
    coop_wave_sync();
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k >= n) break;
      fp2_t& o = k == 0 ? o0 : (k == 1 ? o1 : o2);
      const fp_t p0 = lds_get(&L->P[k][0]), p1 = lds_get(&L->P[k][1]), p2 = lds_get(&L->P[k][2]);
      fp_t w;
      fp_add_sub(w, p0, p1, o.c0, p0, p1);
      fp_sub(o.c1, p2, w);
    }
    coop_wave_sync();
#else
    cg_prod1(S, q, a0, b0, o0);
    if (n > 1) cg_prod1(S, q, a1, b1, o1);
    if (n > 2) cg_prod1(S, q, a2, b2, o2);
#endif
    return;
  }
  const fp2_t a = cg_sel(s, a0, a1, a2), b = cg_sel(s, b0, b1, b2);
  fp_t u, v;
  if (q == 0) {
    u = a.c0;
    v = b.c0;
  } else if (q == 1) {
    u = a.c1;
    v = b.c1;
  } else {
    fp_add_lazy(u, a.c0, a.c1);  // < 2p, product inputs only
    fp_add_lazy(v, b.c0, b.c1);
  }
  fp_t r;
  fp_mul(r, u, v);
#if BGV_CG_SPLIT_COMBINE
  // S always points at the kernel's __shared__ scratch: LDS accesses (lds.h)
  BGV_LDS cg_scratch* L = (BGV_LDS cg_scratch*)S;
  if ((int)s < n) lds_put(&L->P[s][q], r);
  coop_wave_sync();
  // lane (s, 0) forms c0 = P0 - P1 of slot s, lane (s, 1) c1 = P2 - P0 - P1,
  // then every lane reads the n products back: one more LDS exchange
  // instead of 3 x 3 redundant additions on every lane
  if ((int)s < n && q < 2) {
    // both lanes run the same dual add/sub (no divergent branches), then
    // lane 1 finishes c1 = P2 - (P0 + P1)
    const fp_t p0 = lds_get(&L->P[s][0]), p1 = lds_get(&L->P[s][1]);
    fp_t o, w;
    fp_add_sub(w, p0, p1, o, p0, p1);
    if (q == 1) fp_sub(o, lds_get(&L->P[s][2]), w);
    lds_put(&L->O[s][q], o);
  }
  coop_wave_sync();
  o0.c0 = lds_get(&L->O[0][0]);
  o0.c1 = lds_get(&L->O[0][1]);
  if (n > 1) {
    o1.c0 = lds_get(&L->O[1][0]);
    o1.c1 = lds_get(&L->O[1][1]);
  }
  if (n > 2) {
    o2.c0 = lds_get(&L->O[2][0]);
    o2.c1 = lds_get(&L->O[2][1]);
  }
#else
  if ((int)s < n) S->P[s][q] = r;
  coop_wave_sync();
  cg_combine(o0, S->P[0]);
  if (n > 1) cg_combine(o1, S->P[1]);
  if (n > 2) cg_combine(o2, S->P[2]);
#endif
  coop_wave_sync();
}

// dbl-2009-l (curve.h jac_dbl): 3 rounds
template <int SLOTS>
BGV_CGF void cg_dbl(cg_scratch* S, uint32_t s, uint32_t q, g2j& r, const g2j& p) {
  fp2_t A, B, T, C, Sq, F, E, t, D, x3, G, xb;
  cg_round<SLOTS>(S, s, q, 3, p.x, p.x, p.y, p.y, p.y, p.z, A, B, T);
  fp2_dbl(E, A);
  fp2_add(E, E, A);
  fp2_add(xb, p.x, B);
  cg_round<SLOTS>(S, s, q, 3, B, B, xb, xb, E, E, C, Sq, F);
  fp2_sub(t, Sq, A);
  fp2_sub(t, t, C);
  fp2_dbl(D, t);
  fp2_dbl(t, D);
  fp2_sub(x3, F, t);
  fp2_sub(t, D, x3);
  cg_round<SLOTS>(S, s, q, 1, E, t, E, t, E, t, G, G, G);
  fp2_dbl(C, C);
  fp2_dbl(C, C);
  fp2_dbl(C, C);
  fp2_sub(r.y, G, C);
  fp2_dbl(r.z, T);
  r.x = x3;
}

// add-2007-bl with the exceptional cases (curve.h jac_add): 6 rounds
template <int SLOTS>
BGV_CGF void cg_add(cg_scratch* S, uint32_t s, uint32_t q, g2j& r, const g2j& p, const g2j& qq) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(qq);
  fp2_t z1z1, z2z2, zz, u1, u2, a, b, s1, s2, h, h2, i, j, v, rr, x, z3, x3, y, w, t, zs;
  fp2_add(zs, p.z, qq.z);
  cg_round<SLOTS>(S, s, q, 3, p.z, p.z, qq.z, qq.z, zs, zs, z1z1, z2z2, zz);
  cg_round<SLOTS>(S, s, q, 3, p.x, z2z2, qq.x, z1z1, p.y, qq.z, u1, u2, a);
  fp2_sub(h, u2, u1);
  fp2_dbl(h2, h);
  cg_round<SLOTS>(S, s, q, 3, qq.y, p.z, a, z2z2, h2, h2, b, s1, i);
  cg_round<SLOTS>(S, s, q, 3, b, z1z1, h, i, u1, i, s2, j, v);
  fp2_sub(rr, s2, s1);
  const bool h0 = fp2_is_zero(h), r0 = fp2_is_zero(rr);
  fp2_dbl(rr, rr);
  fp2_sub(t, zz, z1z1);
  fp2_sub(t, t, z2z2);
  cg_round<SLOTS>(S, s, q, 2, rr, rr, t, h, t, h, x, z3, z3);
  fp2_sub(x3, x, j);
  fp2_sub(x3, x3, v);
  fp2_sub(x3, x3, v);
  fp2_sub(t, v, x3);
  cg_round<SLOTS>(S, s, q, 2, rr, t, s1, j, s1, j, y, w, w);
  fp2_dbl(w, w);
  g2j sum;
  sum.x = x3;
  fp2_sub(sum.y, y, w);
  sum.z = z3;
  // P == Q: the doubling (rare; every lane of the wave takes the branch
  // together so the rounds inside stay group-wide)
  const bool need_dbl = !pi && !qi && h0 && r0;
  g2j d;
  if (__any(need_dbl)) cg_dbl<SLOTS>(S, s, q, d, p);
  if (pi) r = qq;
  else if (qi) r = p;
  else if (h0) {
    if (r0) r = d;
    else jac_set_inf(r);
  } else r = sum;
}

// [|x|]P (curve.h jac_mul_abs_x): the bits of |x| are wave-uniform
template <int SLOTS>
__device__ void cg_mul_abs_x(cg_scratch* S, uint32_t s, uint32_t q, g2j& r, const g2j& p) {
  g2j acc = p;
  for (int b = 62; b >= 0; b--) {
    cg_dbl<SLOTS>(S, s, q, acc, acc);
    if ((BLS_X_ABS >> b) & 1ull) cg_add<SLOTS>(S, s, q, acc, acc, p);
  }
  r = acc;
}

// [k]P, 4-bit fixed window (curve.h jac_mul_u64_w4); the table (16 points
// per group) sits in LDS
template <int SLOTS>
__device__ void cg_mul_u64_w4(cg_scratch* S, g2j* tab, uint32_t s, uint32_t q, g2j& r, const g2j& p, uint64_t k) {
  const bool lead = s == 0 && q == 0;
  g2j t;
  jac_set_inf(t);
  if (lead) {
    tab[0] = t;
    tab[1] = p;
  }
  cg_dbl<SLOTS>(S, s, q, t, p);
  if (lead) tab[2] = t;
#pragma unroll 1
  for (int i = 3; i < 16; i++) {
    cg_add<SLOTS>(S, s, q, t, t, p);
    if (lead) tab[i] = t;
  }
  coop_wave_sync();
  g2j acc = tab[(k >> 60) & 15];
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    cg_dbl<SLOTS>(S, s, q, acc, acc);
    cg_dbl<SLOTS>(S, s, q, acc, acc);
    cg_dbl<SLOTS>(S, s, q, acc, acc);
    cg_dbl<SLOTS>(S, s, q, acc, acc);
    const g2j e = tab[(k >> (4 * w)) & 15];
    cg_add<SLOTS>(S, s, q, acc, acc, e);
  }
  r = acc;
}

// h_eff [P] (curve.h g2_clear_cofactor)
template <int SLOTS>
__device__ void cg_clear_cofactor(cg_scratch* S, uint32_t s, uint32_t q, g2j& r, const g2j& p) {
  g2j t1, t2, t3, np;
  cg_mul_abs_x<SLOTS>(S, s, q, t1, p);
  jac_neg(t1, t1);  // [x]P
  cg_mul_abs_x<SLOTS>(S, s, q, t2, t1);
  jac_neg(t2, t2);  // [x^2]P
  jac_neg(np, p);
  cg_add<SLOTS>(S, s, q, t3, t1, np);  // [x - 1]P
  g2_psi(t3, t3);
  jac_neg(t1, t1);
  cg_add<SLOTS>(S, s, q, t2, t2, t1);  // [x^2 - x]P
  cg_add<SLOTS>(S, s, q, t2, t2, np);  // [x^2 - x - 1]P
  cg_add<SLOTS>(S, s, q, t2, t2, t3);
  cg_dbl<SLOTS>(S, s, q, t1, p);
  g2_psi2(t1, t1);
  cg_add<SLOTS>(S, s, q, r, t2, t1);
}

// psi(P) == [x]P (curve.h g2_in_subgroup)
template <int SLOTS>
__device__ bool cg_in_subgroup(cg_scratch* S, uint32_t s, uint32_t q, const g2j& p) {
  g2j xp, ps;
  cg_mul_abs_x<SLOTS>(S, s, q, xp, p);
  if (jac_is_inf(p)) return true;
  jac_neg(xp, xp);
  g2_psi(ps, p);
  return jac_eq(ps, xp);
}

}  // namespace bgv
