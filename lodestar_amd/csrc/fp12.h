// Fp6 = Fp2[v] / (v^3 - xi), Fp12 = Fp6[w] / (w^2 - v), xi = 1 + i.
// Coefficient c_k of w^k (k = 0..5) sits at:  k=0 c0.c0, 1 c1.c0, 2 c0.c1,
// 3 c1.c1, 4 c0.c2, 5 c1.c2.  Final exponentiation, cyclotomic squaring and
// Frobenius maps for the pairing check of
// packages/beacon-node/src/chain/bls/maybeBatch.ts:18 (blst finalverify).
#pragma once
#include "fp2.h"

namespace bgv {

#ifndef BGV_FP6_INLINE_FP2
#define BGV_FP6_INLINE_FP2 0
#endif
// code-generation knobs (bgv_kernels.hip / bgv_tail.hip pick per unit)
#if defined(__HIPCC__) && BGV_FP6_INLINE
#define BGV_NI6 BGV_HD
#else
#define BGV_NI6 BGV_NI
#endif
#if defined(__HIPCC__) && BGV_FP12_INLINE
#define BGV_NI12 BGV_HD
#else
#define BGV_NI12 BGV_NI
#endif
#if BGV_FP6_INLINE_FP2
#define F6_MUL fp2_mul_inl
#else
#define F6_MUL fp2_mul
#endif

// ---------------------------------------------------------------- Fp6
BGV_HD void fp6_zero(fp6_t& r) { r.c0 = fp2_zero(); r.c1 = fp2_zero(); r.c2 = fp2_zero(); }
BGV_HD void fp6_one(fp6_t& r) { r.c0 = fp2_one(); r.c1 = fp2_zero(); r.c2 = fp2_zero(); }

BGV_HD void fp6_add(fp6_t& r, const fp6_t& a, const fp6_t& b) {
  fp2_add(r.c0, a.c0, b.c0); fp2_add(r.c1, a.c1, b.c1); fp2_add(r.c2, a.c2, b.c2);
}
BGV_HD void fp6_sub(fp6_t& r, const fp6_t& a, const fp6_t& b) {
  fp2_sub(r.c0, a.c0, b.c0); fp2_sub(r.c1, a.c1, b.c1); fp2_sub(r.c2, a.c2, b.c2);
}
BGV_HD void fp6_neg(fp6_t& r, const fp6_t& a) { fp2_neg(r.c0, a.c0); fp2_neg(r.c1, a.c1); fp2_neg(r.c2, a.c2); }

// r = a * v  (v^3 = xi)
BGV_HD void fp6_mul_v(fp6_t& r, const fp6_t& a) {
  fp2_t t;
  fp2_mul_xi(t, a.c2);
  r.c2 = a.c1;
  r.c1 = a.c0;
  r.c0 = t;
}

// Karatsuba-style, 6 Fp2 products
BGV_NI6 void fp6_mul(fp6_t& r, const fp6_t& a, const fp6_t& b) {
  fp2_t t0, t1, t2, s0, s1, u;
  F6_MUL(t0, a.c0, b.c0);
  F6_MUL(t1, a.c1, b.c1);
  F6_MUL(t2, a.c2, b.c2);
  // c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2)
  fp2_add(s0, a.c1, a.c2);
  fp2_add(s1, b.c1, b.c2);
  F6_MUL(u, s0, s1);
  fp2_sub(u, u, t1);
  fp2_sub(u, u, t2);
  fp2_mul_xi(u, u);
  fp2_t c0;
  fp2_add(c0, u, t0);
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  fp2_add(s0, a.c0, a.c1);
  fp2_add(s1, b.c0, b.c1);
  F6_MUL(u, s0, s1);
  fp2_sub(u, u, t0);
  fp2_sub(u, u, t1);
  fp2_t x2;
  fp2_mul_xi(x2, t2);
  fp2_t c1;
  fp2_add(c1, u, x2);
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  fp2_add(s0, a.c0, a.c2);
  fp2_add(s1, b.c0, b.c2);
  F6_MUL(u, s0, s1);
  fp2_sub(u, u, t0);
  fp2_sub(u, u, t2);
  fp2_add(r.c2, u, t1);
  r.c0 = c0;
  r.c1 = c1;
}

BGV_HD void fp6_sqr(fp6_t& r, const fp6_t& a) { fp6_mul(r, a, a); }

// a * (b0 + b1 v): 5 Fp2 products
BGV_NI6 void fp6_mul_01(fp6_t& r, const fp6_t& a, const fp2_t& b0, const fp2_t& b1) {
  fp2_t t0, t1, u, s0, s1, c0, c1, c2;
  F6_MUL(t0, a.c0, b0);
  F6_MUL(t1, a.c1, b1);
  // c0 = t0 + xi a2 b1
  F6_MUL(u, a.c2, b1);
  fp2_mul_xi(u, u);
  fp2_add(c0, u, t0);
  // c1 = (a0+a1)(b0+b1) - t0 - t1
  fp2_add(s0, a.c0, a.c1);
  fp2_add(s1, b0, b1);
  F6_MUL(u, s0, s1);
  fp2_sub(u, u, t0);
  fp2_sub(c1, u, t1);
  // c2 = t1 + a2 b0
  F6_MUL(u, a.c2, b0);
  fp2_add(c2, u, t1);
  r.c0 = c0; r.c1 = c1; r.c2 = c2;
}

// a * (b1 v): 3 Fp2 products
BGV_NI6 void fp6_mul_1(fp6_t& r, const fp6_t& a, const fp2_t& b1) {
  fp2_t c0, c1, c2;
  F6_MUL(c0, a.c2, b1);
  fp2_mul_xi(c0, c0);
  F6_MUL(c1, a.c0, b1);
  F6_MUL(c2, a.c1, b1);
  r.c0 = c0; r.c1 = c1; r.c2 = c2;
}

// a * (b1 v + b2 v^2): 5 Fp2 products
BGV_NI6 void fp6_mul_12(fp6_t& r, const fp6_t& a, const fp2_t& b1, const fp2_t& b2) {
  fp2_t t1, t2, u, s0, s1, c0, c1, c2;
  F6_MUL(t1, a.c1, b1);
  F6_MUL(t2, a.c2, b2);
  // c0 = xi (a1 b2 + a2 b1) = xi ((a1+a2)(b1+b2) - t1 - t2)
  fp2_add(s0, a.c1, a.c2);
  fp2_add(s1, b1, b2);
  F6_MUL(u, s0, s1);
  fp2_sub(u, u, t1);
  fp2_sub(u, u, t2);
  fp2_mul_xi(c0, u);
  // c1 = a0 b1 + xi t2
  F6_MUL(u, a.c0, b1);
  fp2_mul_xi(t2, t2);
  fp2_add(c1, u, t2);
  // c2 = a0 b2 + t1
  F6_MUL(u, a.c0, b2);
  fp2_add(c2, u, t1);
  r.c0 = c0; r.c1 = c1; r.c2 = c2;
}

BGV_NI void fp6_inv(fp6_t& r, const fp6_t& a) {
  // c0 = a0^2 - xi a1 a2, c1 = xi a2^2 - a0 a1, c2 = a1^2 - a0 a2
  fp2_t c0, c1, c2, t;
  fp2_sqr(c0, a.c0);
  fp2_mul(t, a.c1, a.c2);
  fp2_mul_xi(t, t);
  fp2_sub(c0, c0, t);
  fp2_sqr(c1, a.c2);
  fp2_mul_xi(c1, c1);
  fp2_mul(t, a.c0, a.c1);
  fp2_sub(c1, c1, t);
  fp2_sqr(c2, a.c1);
  fp2_mul(t, a.c0, a.c2);
  fp2_sub(c2, c2, t);
  // n = a0 c0 + xi (a2 c1 + a1 c2)
  fp2_t n, u;
  fp2_mul(n, a.c2, c1);
  fp2_mul(u, a.c1, c2);
  fp2_add(n, n, u);
  fp2_mul_xi(n, n);
  fp2_mul(u, a.c0, c0);
  fp2_add(n, n, u);
  fp2_inv(n, n);
  fp2_mul(r.c0, c0, n);
  fp2_mul(r.c1, c1, n);
  fp2_mul(r.c2, c2, n);
}

// --------------------------------------------------------------- Fp12
BGV_HD void fp12_one(fp12_t& r) { fp6_one(r.c0); fp6_zero(r.c1); }

BGV_HD bool fp12_is_one(const fp12_t& a) {
  return fp2_is_one(a.c0.c0) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}

BGV_HD void fp12_conj(fp12_t& r, const fp12_t& a) { r.c0 = a.c0; fp6_neg(r.c1, a.c1); }

BGV_NI void fp12_mul(fp12_t& r, const fp12_t& a, const fp12_t& b) {
  fp6_t t0, t1, s0, s1;
  fp6_mul(t0, a.c0, b.c0);
  fp6_mul(t1, a.c1, b.c1);
  fp6_add(s0, a.c0, a.c1);
  fp6_add(s1, b.c0, b.c1);
  fp6_mul(s0, s0, s1);
  fp6_sub(s0, s0, t0);
  fp6_sub(r.c1, s0, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}

// complex squaring: (a0 + a1 w)^2 = (a0^2 + v a1^2) + 2 a0 a1 w, 2 Fp6 products
BGV_NI12 void fp12_sqr(fp12_t& r, const fp12_t& a) {
  fp6_t t0, t1, t2;
  fp6_mul(t0, a.c0, a.c1);          // a0 a1
  fp6_add(t1, a.c0, a.c1);          // a0 + a1
  fp6_mul_v(t2, a.c1);              // v a1
  fp6_add(t2, a.c0, t2);            // a0 + v a1
  fp6_mul(t1, t1, t2);              // (a0+a1)(a0+v a1) = a0^2 + v a1^2 + a0a1(1+v)
  fp6_sub(t1, t1, t0);
  fp6_mul_v(t2, t0);
  fp6_sub(r.c0, t1, t2);
  fp6_add(r.c1, t0, t0);
}

// multiply by a sparse line  l = a0 + a1 w^2 + b1 w^3  (tower: c0 = (a0, a1, 0), c1 = (0, b1, 0))
BGV_NI12 void fp12_mul_line(fp12_t& r, const fp12_t& f, const fp2_t& a0, const fp2_t& a1, const fp2_t& b1) {
  fp6_t t0, t1, s;
  fp6_mul_01(t0, f.c0, a0, a1);
  fp6_mul_1(t1, f.c1, b1);
  fp6_add(s, f.c0, f.c1);
  fp2_t a1b1;
  fp2_add(a1b1, a1, b1);
  fp6_mul_01(s, s, a0, a1b1);
  fp6_sub(s, s, t0);
  fp6_sub(r.c1, s, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}

// f * l * l' for two sparse lines l = a0 + a1 w^2 + b1 w^3, l' = c0 + c1 w^2 + d1 w^3
// (the two pairs of one multi-Miller step): the lines are multiplied first,
//   l l' = (a0c0 + xi b1d1, a0c1 + a1c0, a1c1) + (0, a0d1 + b1c0, a1d1 + b1c1) w
// (6 Fp2 products), then f by that five-term element (6 + 5 + 6): 23 Fp2
// products against 26 for two fp12_mul_line, and f is read and written once
BGV_NI12 void fp12_mul_line2(fp12_t& r, const fp12_t& f, const fp2_t& a0, const fp2_t& a1, const fp2_t& b1,
                             const fp2_t& c0, const fp2_t& c1, const fp2_t& d1) {
  fp2_t ac0, ac1, bd, s, u;
  fp6_t x;
  fp2_t y1, y2;
  F6_MUL(ac0, a0, c0);
  F6_MUL(ac1, a1, c1);
  F6_MUL(bd, b1, d1);
  fp2_mul_xi(u, bd);
  fp2_add(x.c0, ac0, u);
  fp2_add(s, a0, a1);
  fp2_add(u, c0, c1);
  F6_MUL(x.c1, s, u);
  fp2_sub(x.c1, x.c1, ac0);
  fp2_sub(x.c1, x.c1, ac1);
  x.c2 = ac1;
  fp2_add(s, a0, b1);
  fp2_add(u, c0, d1);
  F6_MUL(y1, s, u);
  fp2_sub(y1, y1, ac0);
  fp2_sub(y1, y1, bd);
  fp2_add(s, a1, b1);
  fp2_add(u, c1, d1);
  F6_MUL(y2, s, u);
  fp2_sub(y2, y2, ac1);
  fp2_sub(y2, y2, bd);
  // f (x + y w) with y = y1 v + y2 v^2
  fp6_t t0, t1, sf;
  fp6_mul(t0, f.c0, x);
  fp6_mul_12(t1, f.c1, y1, y2);
  fp6_add(sf, f.c0, f.c1);
  fp2_add(x.c1, x.c1, y1);
  fp2_add(x.c2, x.c2, y2);
  fp6_mul(sf, sf, x);
  fp6_sub(sf, sf, t0);
  fp6_sub(r.c1, sf, t1);
  fp6_mul_v(t1, t1);
  fp6_add(r.c0, t0, t1);
}

BGV_NI void fp12_inv(fp12_t& r, const fp12_t& a) {
  // 1 / (a0 + a1 w) = (a0 - a1 w) / (a0^2 - v a1^2)
  fp6_t t0, t1;
  fp6_sqr(t0, a.c0);
  fp6_sqr(t1, a.c1);
  fp6_mul_v(t1, t1);
  fp6_sub(t0, t0, t1);
  fp6_inv(t0, t0);
  fp6_mul(r.c0, a.c0, t0);
  fp6_mul(t1, a.c1, t0);
  fp6_neg(r.c1, t1);
}

// pi^k for k = 1, 2, 3: coefficient at w^i -> conj^k(c_i) * FROB_G[k-1][i-1]
BGV_NI void fp12_frob(fp12_t& r, const fp12_t& a, int k) {
  fp2_t c[6] = {a.c0.c0, a.c1.c0, a.c0.c1, a.c1.c1, a.c0.c2, a.c1.c2};
  if (k & 1) {
#pragma unroll
    for (int i = 0; i < 6; i++) fp2_conj(c[i], c[i]);
  }
#pragma unroll
  for (int i = 1; i < 6; i++) fp2_mul(c[i], c[i], FROB_G[k - 1][i - 1]);
  r.c0.c0 = c[0]; r.c1.c0 = c[1]; r.c0.c1 = c[2]; r.c1.c1 = c[3]; r.c0.c2 = c[4]; r.c1.c2 = c[5];
}

// (a + b s)^2 in Fp4 = Fp2[s]/(s^2 - xi)
BGV_NI void fp4_sqr(fp2_t& r0, fp2_t& r1, const fp2_t& a, const fp2_t& b) {
  fp2_t t0, t1, t2;
  fp2_sqr(t0, a);
  fp2_sqr(t1, b);
  fp2_mul_xi(t2, t1);
  fp2_add(r0, t2, t0);
  fp2_add(t2, a, b);
  fp2_sqr(t2, t2);
  fp2_sub(t2, t2, t0);
  fp2_sub(r1, t2, t1);
}

// Granger-Scott squaring, valid in the cyclotomic subgroup (after the easy part).
// Fp12 viewed as Fp4[t]/(t^3 - s), s = w^3: A = c0 + c3 s, B = c1 + c4 s, C = c2 + c5 s.
// A' = 3A^2 - 2 conj(A), B' = 3 s C^2 + 2 conj(B), C' = 3B^2 - 2 conj(C).
BGV_NI void fp12_cyclotomic_sqr(fp12_t& r, const fp12_t& f) {
  fp2_t z0 = f.c0.c0, z1 = f.c1.c1;  // A
  fp2_t z2 = f.c1.c0, z3 = f.c0.c2;  // B
  fp2_t z4 = f.c0.c1, z5 = f.c1.c2;  // C
  fp2_t t0, t1, t2, t3, u;
  fp4_sqr(t0, t1, z0, z1);
  fp2_sub(u, t0, z0); fp2_dbl(u, u); fp2_add(z0, u, t0);
  fp2_add(u, t1, z1); fp2_dbl(u, u); fp2_add(z1, u, t1);
  fp4_sqr(t0, t1, z2, z3);
  fp4_sqr(t2, t3, z4, z5);
  fp2_sub(u, t0, z4); fp2_dbl(u, u); fp2_add(z4, u, t0);
  fp2_add(u, t1, z5); fp2_dbl(u, u); fp2_add(z5, u, t1);
  fp2_mul_xi(t0, t3);
  fp2_add(u, t0, z2); fp2_dbl(u, u); fp2_add(z2, u, t0);
  fp2_sub(u, t2, z3); fp2_dbl(u, u); fp2_add(z3, u, t2);
  r.c0.c0 = z0; r.c1.c1 = z1; r.c1.c0 = z2; r.c0.c2 = z3; r.c0.c1 = z4; r.c1.c2 = z5;
}

// r = a^x for the (negative) BLS parameter x, a in the cyclotomic subgroup
BGV_NI void fp12_pow_x(fp12_t& r, const fp12_t& a) {
  fp12_t acc = a;
  for (int b = 62; b >= 0; b--) {
    fp12_cyclotomic_sqr(acc, acc);
    if ((BLS_X_ABS >> b) & 1ull) fp12_mul(acc, acc, a);
  }
  fp12_conj(r, acc);  // x < 0
}

// f^((p^12 - 1) / r) up to the fixed cube: the hard part uses
// 3 (p^4 - p^2 + 1) / r = (x - 1)^2 (x + p)(x^2 + p^2 - 1) + 3.
// Equality with 1 is unaffected by the cube (gcd(3, r) = 1).
BGV_NI void fp12_final_exp(fp12_t& r, const fp12_t& f) {
  fp12_t t0, t1, y0, y1, y2, y3;
  // easy part: f^((p^6 - 1)(p^2 + 1))
  fp12_inv(t0, f);
  fp12_conj(t1, f);
  fp12_mul(t1, t1, t0);     // f^(p^6 - 1)
  fp12_frob(t0, t1, 2);
  fp12_mul(t1, t0, t1);     // m = f^((p^6-1)(p^2+1))
  // hard part
  fp12_pow_x(t0, t1);
  fp12_conj(y0, t1);
  fp12_mul(y0, t0, y0);     // m^(x-1)
  fp12_pow_x(t0, y0);
  fp12_conj(y1, y0);
  fp12_mul(y1, t0, y1);     // m^((x-1)^2)
  fp12_pow_x(t0, y1);
  fp12_frob(y2, y1, 1);
  fp12_mul(y2, t0, y2);     // y1^(x + p)
  fp12_pow_x(t0, y2);
  fp12_pow_x(t0, t0);       // y2^(x^2)
  fp12_frob(y3, y2, 2);
  fp12_mul(y3, t0, y3);
  fp12_conj(t0, y2);
  fp12_mul(y3, y3, t0);     // y2^(x^2 + p^2 - 1)
  fp12_cyclotomic_sqr(t0, t1);
  fp12_mul(t0, t0, t1);     // m^3
  fp12_mul(r, y3, t0);
}

}  // namespace bgv
