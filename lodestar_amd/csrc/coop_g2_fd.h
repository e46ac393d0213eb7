// Cooperative G2 point arithmetic of the latency mode over the signed-digit
// field (fd.h): TWELVE lanes per point.  Every lane of a group holds the
// whole point and runs the additions redundantly (carry-free digit-wise
// operations); only the Fp2 products are distributed: a round computes up
// to three Fp2 products, lane (s, q) (slot s = 0..2, q = 0..3) one Fp
// product of the schoolbook  a0 b0 | a1 b1 | a0 b1 | a1 b0, exchanged
// through LDS inside one wave; every lane then forms c0 = P0 - P1,
// c1 = P2 + P3 itself.  (Schoolbook rather than Karatsuba: no operand sums,
// so a product's value bound is that of its inputs.)  A doubling is 3
// rounds, an addition 6.
//
// Formulas and their order are those of curve.h (dbl-2009-l, add-2007-bl
// with the exceptional cases, the 4-bit fixed window of jac_mul_u64_w4, the
// x-chain of jac_mul_abs_x, Budroni-Pintore h_eff, Scott's subgroup test), so
// the points are the one-lane kernels' as field elements (GPU test: latency
// mode on/off).  The formulas are templates over the product round, so the
// host build runs them one lane at a time under the fd bound checks
// (tests/native/fdcheck.cpp).
//
// Bounds (V = |value| / p, digits in units of 2^28; fd.h):
//   point coordinates between operations: digits normalized, V <= 8.8;
//   a round's products: digits <= 2^59 and V_a V_b <= 252 (each commented),
//   outputs: c0 digits in (-2^28, 2^28), c1 in [0, 2^29), V <= 2.2.
#pragma once
#include "fd.h"
#include "curve.h"
#if defined(__HIPCC__)
#include "lds.h"
#endif

namespace bgv {

struct gd2j { fd2_t x, y, z; };

// the doubling and the addition are compiled once each (their fd2
// temporaries allocated per function); everything above them inlines them
#if defined(__HIPCC__)
#define GD_NI __device__ __noinline__
#else
#define GD_NI static inline
#endif

constexpr int GD_LANES = 12;
constexpr int GD_GROUPS = 64 / GD_LANES;  // 5 points per wave

// ---- product rounds ---------------------------------------------------------
// host: the products of a round one after another on this lane
struct gd_host {
  BGV_HD void prod(fd2_t& o, const fd2_t& a, const fd2_t& b) {
    fd_t p0, p1, p2, p3;
    fd_mul(p0, a.c0, b.c0);
    fd_mul(p1, a.c1, b.c1);
    fd_mul(p2, a.c0, b.c1);
    fd_mul(p3, a.c1, b.c0);
    fd_sub(o.c0, p0, p1);
    fd_add(o.c1, p2, p3);
  }
  BGV_HD void round(int n, const fd2_t& a0, const fd2_t& b0, const fd2_t& a1, const fd2_t& b1, const fd2_t& a2,
                    const fd2_t& b2, fd2_t& o0, fd2_t& o1, fd2_t& o2) {
    fd2_t r0, r1, r2;
    prod(r0, a0, b0);
    if (n > 1) prod(r1, a1, b1);
    if (n > 2) prod(r2, a2, b2);
    o0 = r0;
    if (n > 1) o1 = r1;
    if (n > 2) o2 = r2;
  }
  BGV_HD void sync() {}
};

#if defined(__HIPCC__)
struct gd_scratch {
  fd_t P[3][4];  // [slot][schoolbook product]
};

__device__ __forceinline__ fd_t lds_get_fd(const BGV_LDS fd_t* p) {
  fd_t r;
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = p->d[k];
  return r;
}
__device__ __forceinline__ void lds_put_fd(BGV_LDS fd_t* p, const fd_t& v) {
#pragma unroll
  for (int k = 0; k < ND; k++) p->d[k] = v.d[k];
}

// device: lane (s, q) of a 12-lane group; S is the group's __shared__ scratch
struct gd_dev {
  gd_scratch* S;
  uint32_t s, q;
  __device__ __forceinline__ void sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
  __device__ __forceinline__ void round(int n, const fd2_t& a0, const fd2_t& b0, const fd2_t& a1, const fd2_t& b1,
                                        const fd2_t& a2, const fd2_t& b2, fd2_t& o0, fd2_t& o1, fd2_t& o2) {
    const fd2_t a = s == 0 ? a0 : (s == 1 ? a1 : a2);
    const fd2_t b = s == 0 ? b0 : (s == 1 ? b1 : b2);
    const fd_t u = (q == 0 || q == 2) ? a.c0 : a.c1;
    const fd_t v = (q == 0 || q == 3) ? b.c0 : b.c1;
    fd_t r;
    fd_mul(r, u, v);
    BGV_LDS gd_scratch* L = (BGV_LDS gd_scratch*)S;
    if ((int)s < n) lds_put_fd(&L->P[s][q], r);
    sync();
    fd_sub(o0.c0, lds_get_fd(&L->P[0][0]), lds_get_fd(&L->P[0][1]));
    fd_add(o0.c1, lds_get_fd(&L->P[0][2]), lds_get_fd(&L->P[0][3]));
    if (n > 1) {
      fd_sub(o1.c0, lds_get_fd(&L->P[1][0]), lds_get_fd(&L->P[1][1]));
      fd_add(o1.c1, lds_get_fd(&L->P[1][2]), lds_get_fd(&L->P[1][3]));
    }
    if (n > 2) {
      fd_sub(o2.c0, lds_get_fd(&L->P[2][0]), lds_get_fd(&L->P[2][1]));
      fd_add(o2.c1, lds_get_fd(&L->P[2][2]), lds_get_fd(&L->P[2][3]));
    }
    sync();
  }
};
#endif

// ---- points -----------------------------------------------------------------
BGV_HD bool gd_is_inf(const gd2j& p) { return fd2_is_zero(p.z); }
BGV_HD void gd_set_inf(gd2j& p) { p.x = fd2_one(); p.y = fd2_one(); p.z = fd2_zero(); }
BGV_HD void gd_neg(gd2j& r, const gd2j& p) { r.x = p.x; fd2_neg(r.y, p.y); r.z = p.z; }

// dbl-2009-l (curve.h jac_dbl)
template <class RP> GD_NI void gd_dbl(RP rp, gd2j& r, const gd2j& p) {
  fd2_t A, B, T, E, xb, C, Sq, F, t, D, t2, x3, t3, G, C2, y3, z3;
  rp.round(3, p.x, p.x, p.y, p.y, p.y, p.z, A, B, T);  // X^2, Y^2, YZ (V <= 77)
  fd2_norm(B, B);
  fd2_mulc<3>(E, A);
  fd2_norm(E, E);                                      // E = 3A: V 6.6
  fd2_add(xb, p.x, B);                                 // V <= 11, digits 2x
  rp.round(3, B, B, xb, xb, E, E, C, Sq, F);           // C = B^2, (X+B)^2 (V 121), F = E^2
  fd2_sub(t, Sq, A);
  fd2_sub(t, t, C);
  fd2_norm(t, t);
  fd2_dbl(D, t);
  fd2_fold(D, D);                                      // D = 2((X+B)^2 - A - C): V 0.6
  fd2_dbl(t2, D);
  fd2_sub(x3, F, t2);                                  // X3 = F - 2D: V 3.4
  fd2_sub(t3, D, x3);                                  // V 4.0, digits < 2^30.3
  rp.round(1, E, t3, E, t3, E, t3, G, G, G);           // G = E (D - X3): V 26
  fd2_dbl(C2, C);
  fd2_norm(C2, C2);
  fd2_mulc<4>(C2, C2);
  fd2_sub(y3, G, C2);
  fd2_fold(y3, y3);                                    // Y3 = G - 8C: V 0.6
  fd2_dbl(z3, T);
  fd2_norm(z3, z3);                                    // Z3 = 2YZ: V 4.4
  fd2_norm(x3, x3);
  r.x = x3;
  r.y = y3;
  r.z = z3;
}

// add-2007-bl with the exceptional cases (curve.h jac_add)
template <class RP> GD_NI void gd_add(RP rp, gd2j& r, const gd2j& p, const gd2j& qq) {
  const bool pi = gd_is_inf(p), qi = gd_is_inf(qq);
  fd2_t zs, z1z1, z2z2, zz, u1, u2, a, h, h2, b, s1, i, s2, j, v, rr, t, x, z3, x3, y, w, y3;
  fd2_add(zs, p.z, qq.z);
  fd2_fold(zs, zs);
  rp.round(3, p.z, p.z, qq.z, qq.z, zs, zs, z1z1, z2z2, zz);  // V <= 77
  rp.round(3, p.x, z2z2, qq.x, z1z1, p.y, qq.z, u1, u2, a);   // V <= 19, 19, 77
  fd2_sub(h, u2, u1);
  fd2_norm(h, h);                                              // V 4.4
  fd2_dbl(h2, h);                                              // V 8.8, digits 2x
  rp.round(3, qq.y, p.z, a, z2z2, h2, h2, b, s1, i);           // V 77, 4.8, 77
  rp.round(3, b, z1z1, h, i, u1, i, s2, j, v);                 // V 4.8, 9.7, 4.8
  fd2_sub(rr, s2, s1);
  fd2_norm(rr, rr);                                            // V 4.4
  const bool h0 = fd2_is_zero(h), r0 = fd2_is_zero(rr);
  fd2_dbl(rr, rr);                                             // V 8.8
  fd2_sub(t, zz, z1z1);
  fd2_sub(t, t, z2z2);
  fd2_norm(t, t);                                              // V 6.6
  rp.round(2, rr, rr, t, h, t, h, x, z3, z3);                  // V 77, 29
  fd2_sub(x3, x, j);
  fd2_norm(x3, x3);
  fd2_sub(x3, x3, v);
  fd2_sub(x3, x3, v);                                          // X3 = rr^2 - j - 2v: V 8.8
  fd2_sub(t, v, x3);
  fd2_norm(t, t);                                              // V 11
  rp.round(2, rr, t, s1, j, s1, j, y, w, w);                   // V 97, 4.8
  fd2_dbl(w, w);
  fd2_sub(y3, y, w);                                           // V 6.6
  gd2j sum;
  fd2_norm(sum.x, x3);
  fd2_norm(sum.y, y3);
  fd2_norm(sum.z, z3);
  // P == Q: the doubling (rare; every lane of the wave takes the branch together)
  const bool need_dbl = !pi && !qi && h0 && r0;
  gd2j d;
#if defined(__HIP_DEVICE_COMPILE__)
  if (__any(need_dbl)) gd_dbl(rp, d, p);
#else
  if (need_dbl) gd_dbl(rp, d, p);
#endif
  if (pi) r = qq;
  else if (qi) r = p;
  else if (h0) {
    if (r0) r = d;
    else gd_set_inf(r);
  } else r = sum;
}

// [|x|]P (curve.h jac_mul_abs_x)
template <class RP> BGV_HD void gd_mul_abs_x(RP rp, gd2j& r, const gd2j& p) {
  gd2j acc = p;
  for (int b = 62; b >= 0; b--) {
    gd_dbl(rp, acc, acc);
    if ((BLS_X_ABS >> b) & 1ull) gd_add(rp, acc, acc, p);
  }
  r = acc;
}

// psi (curve.h g2_psi): conj(x) PSI_CX, conj(y) PSI_CY, conj(z)
template <class RP> BGV_HD void gd_psi(RP rp, gd2j& r, const gd2j& p) {
  fd2_t x, y, z, ox, oy;
  fd2_conj(x, p.x);
  fd2_conj(y, p.y);
  fd2_conj(z, p.z);
  rp.round(2, x, FD_PSI_CX, y, FD_PSI_CY, y, FD_PSI_CY, ox, oy, oy);
  fd2_norm(r.x, ox);
  fd2_norm(r.y, oy);
  r.z = z;
}

// psi^2 (curve.h g2_psi2): x PSI2_CX, y PSI2_CY (Fp constants as (c, 0))
template <class RP> BGV_HD void gd_psi2(RP rp, gd2j& r, const gd2j& p) {
  fd2_t cx, cy, ox, oy;
  cx.c0 = FD_PSI2_CX;
  fd_zero(cx.c1);
  cy.c0 = FD_PSI2_CY;
  fd_zero(cy.c1);
  rp.round(2, p.x, cx, p.y, cy, p.y, cy, ox, oy, oy);
  fd2_norm(r.x, ox);
  fd2_norm(r.y, oy);
  r.z = p.z;
}

// h_eff [P] (curve.h g2_clear_cofactor)
template <class RP> BGV_HD void gd_clear_cofactor(RP rp, gd2j& r, const gd2j& p) {
  gd2j t1, t2, t3, np;
  gd_mul_abs_x(rp, t1, p);
  gd_neg(t1, t1);  // [x]P
  gd_mul_abs_x(rp, t2, t1);
  gd_neg(t2, t2);  // [x^2]P
  gd_neg(np, p);
  gd_add(rp, t3, t1, np);  // [x - 1]P
  gd_psi(rp, t3, t3);
  gd_neg(t1, t1);
  gd_add(rp, t2, t2, t1);  // [x^2 - x]P
  gd_add(rp, t2, t2, np);  // [x^2 - x - 1]P
  gd_add(rp, t2, t2, t3);
  gd_dbl(rp, t1, p);
  gd_psi2(rp, t1, t1);
  gd_add(rp, r, t2, t1);
}

// equality of Jacobian points (curve.h jac_eq), cross-multiplied
template <class RP> BGV_HD bool gd_eq(RP rp, const gd2j& p, const gd2j& q) {
  const bool pi = gd_is_inf(p), qi = gd_is_inf(q);
  fd2_t z1z1, z2z2, a, b, t1, t2, c, d, e;
  rp.round(3, p.z, p.z, q.z, q.z, p.y, q.z, z1z1, z2z2, t1);   // V <= 77
  rp.round(3, p.x, z2z2, q.x, z1z1, q.y, p.z, a, b, t2);       // V <= 19, 77
  fd2_norm(t1, t1);
  fd2_norm(t2, t2);
  rp.round(2, t1, z2z2, t2, z1z1, t2, z1z1, c, d, d);          // V 4.8
  fd2_sub(e, a, b);
  const bool xe = fd2_is_zero(e);
  fd2_sub(e, c, d);
  const bool ye = fd2_is_zero(e);
  if (pi || qi) return pi && qi;
  return xe && ye;
}

// psi(P) == [x]P (curve.h g2_in_subgroup)
template <class RP> BGV_HD bool gd_in_subgroup(RP rp, const gd2j& p) {
  gd2j xp, ps;
  gd_mul_abs_x(rp, xp, p);
  const bool inf = gd_is_inf(p);
  gd_neg(xp, xp);
  gd_psi(rp, ps, p);
  const bool eq = gd_eq(rp, ps, xp);
  return inf || eq;
}

// [k]P, 4-bit fixed window (curve.h jac_mul_u64_w4); the 16-point table per
// group sits in LDS on the device (written by the group's lead lane)
template <class RP> BGV_HD void gd_mul_u64_w4(RP rp, gd2j* tab, bool lead, gd2j& r, const gd2j& p, uint64_t k) {
  gd2j t;
  gd_set_inf(t);
  if (lead) {
    tab[0] = t;
    tab[1] = p;
  }
  gd_dbl(rp, t, p);
  if (lead) tab[2] = t;
#pragma unroll 1
  for (int i = 3; i < 16; i++) {
    gd_add(rp, t, t, p);
    if (lead) tab[i] = t;
  }
  rp.sync();
  gd2j acc = tab[(k >> 60) & 15];
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    gd_dbl(rp, acc, acc);
    gd_dbl(rp, acc, acc);
    gd_dbl(rp, acc, acc);
    gd_dbl(rp, acc, acc);
    const gd2j e = tab[(k >> (4 * w)) & 15];
    gd_add(rp, acc, acc, e);
  }
  r = acc;
}

// ---- conversions from / to the fp.h points (rounds with the constants) ------
BGV_HD void fd_digits_of_fp(fd_t& t, const fp_t& a) {
#pragma unroll
  for (int k = 0; k < ND; k++) {
    const int pos = 28 * k, w = pos >> 5, sh = pos & 31;
    const uint32_t lo = w < NL ? a.l[w] : 0u;
    const uint32_t hi = (w + 1) < NL ? a.l[w + 1] : 0u;
    const uint32_t v = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    t.d[k] = (int32_t)(v & (uint32_t)FD_M);
  }
}
BGV_HD void fd2_digits_of_fp2(fd2_t& t, const fp2_t& a) { fd_digits_of_fp(t.c0, a.c0); fd_digits_of_fp(t.c1, a.c1); }

// canonical digits (fd_canon of a conversion product) packed to 12 x u32
BGV_HD void fd_pack_fp(fp_t& r, const fd_t& a) {
  fd_t c;
  fd_canon(c, a);
#pragma unroll
  for (int m = 0; m < NL; m++) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < ND; k++) {
      const int rel = 28 * k - 32 * m;
      if (rel >= 32 || rel <= -28) continue;
      v |= rel >= 0 ? ((uint32_t)c.d[k] << rel) : ((uint32_t)c.d[k] >> (-rel));
    }
    r.l[m] = v;
  }
}

template <class RP> BGV_HD void gd_from_g2j(RP rp, gd2j& r, const g2j& p) {
  fd2_t x, y, z, cin;
  fd2_digits_of_fp2(x, p.x);
  fd2_digits_of_fp2(y, p.y);
  fd2_digits_of_fp2(z, p.z);
  cin.c0 = FD_C_IN;
  fd_zero(cin.c1);
  rp.round(3, x, cin, y, cin, z, cin, r.x, r.y, r.z);  // V 2.2
  fd2_norm(r.x, r.x);
  fd2_norm(r.y, r.y);
  fd2_norm(r.z, r.z);
}

template <class RP> BGV_HD void gd_from_g2a(RP rp, gd2j& r, const g2a& p) {
  fd2_t x, y, cin;
  fd2_digits_of_fp2(x, p.x);
  fd2_digits_of_fp2(y, p.y);
  cin.c0 = FD_C_IN;
  fd_zero(cin.c1);
  rp.round(2, x, cin, y, cin, y, cin, r.x, r.y, r.y);
  fd2_norm(r.x, r.x);
  fd2_norm(r.y, r.y);
  r.z = fd2_one();
}

// the point as canonical fp.h Jacobian coordinates (every lane)
template <class RP> BGV_HD void gd_to_g2j(RP rp, g2j& r, const gd2j& p) {
  fd2_t cout, x, y, z;
  cout.c0 = FD_C_OUT;
  fd_zero(cout.c1);
  rp.round(3, p.x, cout, p.y, cout, p.z, cout, x, y, z);  // V <= 2.2 < the canon range
  fd_pack_fp(r.x.c0, x.c0);
  fd_pack_fp(r.x.c1, x.c1);
  fd_pack_fp(r.y.c0, y.c0);
  fd_pack_fp(r.y.c1, y.c1);
  fd_pack_fp(r.z.c0, z.c0);
  fd_pack_fp(r.z.c1, z.c1);
}

}  // namespace bgv
