// Cooperative G1 arithmetic for the latency mode: three lanes per point.
// Every lane of a group holds the whole point (Fp coordinates) and runs the
// additions of the formulas redundantly; the Fp products of a round go one
// per lane (slot s computes product s) and are exchanged through LDS inside
// one wave.  A doubling (dbl-2009-l) is 3 rounds of one product instead of 7
// products in a row, an addition (add-2007-bl) 6 instead of 16, so the
// [r_i] PK_i multiplication of k_pk (60 doublings, 15 additions after a
// 16-entry table) runs at ~2.5x lower latency on mid-size and small batches,
// where its one-lane form heads the path to the Miller loop.
// Points in Jacobian coordinates as curve.h; the affine results (the only
// values that leave the kernel) are canonical.
#pragma once
#include "miller_coop.h"
#include "lds.h"

namespace bgv {

struct g1c_scratch {
  alignas(16) fp_t O[3];
};

struct g1c_grp {
  g1c_scratch* sc;
  uint32_t s;
};

// o_k = a_k * b_k for k < n (n <= 3): slot s computes product s
__device__ __forceinline__ void g1c_round(const g1c_grp& g, int n, const fp_t& a0, const fp_t& b0, const fp_t& a1,
                                          const fp_t& b1, const fp_t& a2, const fp_t& b2, fp_t& o0, fp_t& o1,
                                          fp_t& o2) {
  BGV_LDS g1c_scratch* L = (BGV_LDS g1c_scratch*)g.sc;
  const fp_t a = g.s == 0 ? a0 : (g.s == 1 ? a1 : a2), b = g.s == 0 ? b0 : (g.s == 1 ? b1 : b2);
  fp_t r;
  fp_mul(r, a, b);
  if ((int)g.s < n) lds_put(&L->O[g.s], r);
  coop_wave_sync();
  o0 = lds_get(&L->O[0]);
  if (n > 1) o1 = lds_get(&L->O[1]);
  if (n > 2) o2 = lds_get(&L->O[2]);
  coop_wave_sync();
}

// dbl-2009-l (curve.h jac_dbl): rounds {X^2, Y^2, YZ}, {B^2, (X + B)^2, E^2}, {E (D - X3)}
__device__ __forceinline__ void g1c_dbl(const g1c_grp& g, g1j& r, const g1j& p) {
  fp_t A, B, T, C, Sq, Fq, E, t, D, x3, y3, xb, c2, d;
  g1c_round(g, 3, p.x, p.x, p.y, p.y, p.y, p.z, A, B, T);
  fp_add2(E, A, A, xb, p.x, B);
  fp_add(E, E, A);  // 3A
  g1c_round(g, 3, B, B, xb, xb, E, E, C, Sq, Fq);
  fp_add_sub(c2, C, C, t, Sq, A);
  fp_add_sub(c2, c2, c2, t, t, C);
  fp_add2(c2, c2, c2, D, t, t);  // 8C, D = 2 (Sq - A - C)
  fp_add2(t, D, D, d, T, T);     // 2D, Z3 = 2YZ
  fp_sub(x3, Fq, t);
  fp_sub(t, D, x3);
  g1c_round(g, 1, E, t, E, t, E, t, y3, y3, y3);
  fp_sub(r.y, y3, c2);
  r.z = d;
  r.x = x3;
}

// add-2007-bl with the exceptional cases (curve.h jac_add); every lane holds
// the values, so the zero tests are local (the wave takes a branch together
// only when a lane needs the doubling)
__device__ __forceinline__ void g1c_add(const g1c_grp& g, g1j& r, const g1j& p, const g1j& q) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  fp_t z1z1, z2z2, zz, u1, u2, a, b, s1, s2, h, h2, i, j, v, rr, x, z3, x3, y, w, t, zs;
  fp_add(zs, p.z, q.z);
  g1c_round(g, 3, p.z, p.z, q.z, q.z, zs, zs, z1z1, z2z2, zz);
  g1c_round(g, 3, p.x, z2z2, q.x, z1z1, p.y, q.z, u1, u2, a);
  fp_sub(h, u2, u1);
  fp_dbl(h2, h);
  g1c_round(g, 3, q.y, p.z, a, z2z2, h2, h2, b, s1, i);
  g1c_round(g, 3, b, z1z1, h, i, u1, i, s2, j, v);
  fp_sub2(rr, s2, s1, t, zz, z1z1);
  const bool h0 = fp_is_zero(h), r0 = fp_is_zero(rr);
  fp_add_sub(rr, rr, rr, t, t, z2z2);
  g1c_round(g, 2, rr, rr, t, h, t, h, x, z3, z3);
  fp_sub(x3, x, j);
  fp_sub(x3, x3, v);
  fp_sub(x3, x3, v);
  fp_sub(t, v, x3);
  g1c_round(g, 2, rr, t, s1, j, s1, j, y, w, w);
  fp_dbl(w, w);
  g1j sum;
  sum.x = x3;
  fp_sub(sum.y, y, w);
  sum.z = z3;
  const bool need_dbl = !pi && !qi && h0 && r0;
  g1j d;
  if (__any(need_dbl)) g1c_dbl(g, d, p);
  if (pi) r = q;
  else if (qi) r = p;
  else if (h0) {
    if (r0) r = d;
    else jac_set_inf(r);
  } else r = sum;
}

// [k]P, 4-bit fixed window (curve.h jac_mul_u64_w4); the 16-entry table sits
// in LDS (written by slot 0, read by every lane); lead = the group owns tab
__device__ void g1c_mul_u64_w4(const g1c_grp& g, g1j* tab, bool lead, g1j& r, const g1j& p, uint64_t k) {
  BGV_LDS g1j* T = (BGV_LDS g1j*)tab;
  const bool wr = lead && g.s == 0;
  auto put = [&](int i, const g1j& v) {
    if (wr) {
      lds_put(&T[i].x, v.x);
      lds_put(&T[i].y, v.y);
      lds_put(&T[i].z, v.z);
    }
  };
  auto get = [&](uint32_t i) {
    g1j v;
    v.x = lds_get(&T[i].x);
    v.y = lds_get(&T[i].y);
    v.z = lds_get(&T[i].z);
    return v;
  };
  g1j t;
  jac_set_inf(t);
  put(0, t);
  put(1, p);
  g1c_dbl(g, t, p);
  put(2, t);
#pragma unroll 1
  for (int i = 3; i < 16; i++) {
    g1c_add(g, t, t, p);
    put(i, t);
  }
  coop_wave_sync();
  g1j acc = get((uint32_t)(k >> 60) & 15u);
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    g1c_dbl(g, acc, acc);
    g1c_dbl(g, acc, acc);
    g1c_dbl(g, acc, acc);
    g1c_dbl(g, acc, acc);
    const g1j e = get((uint32_t)(k >> (4 * w)) & 15u);
    g1c_add(g, acc, acc, e);
  }
  r = acc;
}

}  // namespace bgv
