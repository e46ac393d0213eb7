// Optimal-ate Miller loop for BLS12-381 (loop over |x| = 0xd201000000010000).
// Q in G2 is walked in homogeneous projective coordinates on the M-type
// twist; each line is evaluated at P in G1 (affine) as the sparse element
//   l = a0 + a1 w^2 + b1 w^3
// (line scaled by Fp2 factors / w^3, all of which die in the final
// exponentiation).  Re-creates blst's miller_loop_n used by
// Pairing::commit/finalverify (packages/beacon-node/src/chain/bls/maybeBatch.ts:18).
#pragma once
#include "h2c.h"

#if defined(__HIPCC__) && BGV_STEP_INLINE
#define BGV_NIS BGV_HD
#else
#define BGV_NIS BGV_NI
#endif
// the two-pair loop inlined into its kernel (BGV_LOOP2_INLINE): a __shared__
// accumulator is then seen as LDS by every inlined helper (ds_read/ds_write
// instead of flat accesses)
#if defined(__HIPCC__) && BGV_LOOP2_INLINE
#define BGV_NIL BGV_HD
#else
#define BGV_NIL BGV_NI
#endif
// the two-pair loops multiply each step's two lines together before f
// (fp12_mul_line2: 23 Fp2 products per step instead of 26)
#ifndef BGV_MILLER_LINE2
#define BGV_MILLER_LINE2 1
#endif

namespace bgv {

struct g2p_t { fp2_t x, y, z; };  // homogeneous projective: x = X/Z, y = Y/Z

// r = 3b' a with b' = 4(1+i) (the twist E2: y^2 = x^3 + 4(1+i)): xi-multiply,
// then x4 and x3 by additions instead of a product by the constant
BGV_HD void fp2_mul_3b(fp2_t& r, const fp2_t& a) {
  fp2_t t;
  fp2_mul_xi(t, a);
  fp2_dbl(t, t);
  fp2_dbl(t, t);
  fp2_mul3(r, t);
}

// T <- 2T, line tangent at T evaluated at P.  With AT_P false the line is
// left unevaluated (fixed-argument form, BGV_LINES): a1 = 3X^2 and b1 = 2YZ,
// and miller_line_at_p applies the same P factors later.
template <bool AT_P>
BGV_HD void miller_dbl_core(g2p_t& T, fp2_t& a0, fp2_t& a1, fp2_t& b1, const fp_t& xp, const fp_t& yp) {
  fp2_t A, B, C, E, F, G, H, t;
  fp2_mul(A, T.x, T.y);
  fp_half(A.c0, A.c0);
  fp_half(A.c1, A.c1);           // A = XY/2
  fp2_sqr(B, T.y);               // Y^2
  fp2_sqr(C, T.z);               // Z^2
  fp2_mul_3b(E, C);              // 3b' Z^2 (additions: 3b' = 12(1+i))
  fp2_mul3(F, E);                // 9b' Z^2
  fp2_add(t, T.y, T.z);
  fp2_sqr(t, t);
  fp2_add(H, B, C);
  fp2_sub(H, t, H);              // 2YZ
  // line (negated overall): (3b'Z^2 - Y^2) + 3X^2 xP w^2 - 2YZ yP w^3
  fp2_sub(a0, E, B);
  fp2_sqr(t, T.x);
  fp2_mul3(t, t);
  if constexpr (AT_P) {
    fp2_mul_fp(a1, t, xp);
    fp2_mul_fp(t, H, yp);
    fp2_neg(b1, t);
  } else {
    a1 = t;
    b1 = H;
  }
  // point
  fp2_sub(t, B, F);
  fp2_mul(T.x, A, t);            // X3 = XY/2 (Y^2 - 9b'Z^2)
  fp2_add(G, B, F);
  fp_half(G.c0, G.c0);
  fp_half(G.c1, G.c1);           // (Y^2 + 9b'Z^2)/2
  fp2_sqr(G, G);
  fp2_sqr(t, E);
  fp2_mul3(t, t);                // 27 b'^2 Z^4
  fp2_sub(T.y, G, t);
  fp2_mul(T.z, B, H);            // Z3 = 2 Y^3 Z
}
BGV_NIS void miller_dbl_step(g2p_t& T, fp2_t& a0, fp2_t& a1, fp2_t& b1, const fp_t& xp, const fp_t& yp) {
  miller_dbl_core<true>(T, a0, a1, b1, xp, yp);
}

// T <- T + Q (Q affine), line through T and Q evaluated at P (AT_P false:
// a1 = theta, b1 = lambda, for miller_line_at_p)
template <bool AT_P>
BGV_HD void miller_add_core(g2p_t& T, fp2_t& a0, fp2_t& a1, fp2_t& b1, const g2a& Q,
                                                const fp_t& xp, const fp_t& yp) {
  fp2_t th, la, C, D, E, F, G, H, t;
  fp2_mul(t, Q.y, T.z);
  fp2_sub(th, T.y, t);           // theta = Y - yQ Z
  fp2_mul(t, Q.x, T.z);
  fp2_sub(la, T.x, t);           // lambda = X - xQ Z
  // line: (theta xQ - lambda yQ) - theta xP w^2 + lambda yP w^3
  fp2_mul(a0, th, Q.x);
  fp2_mul(t, la, Q.y);
  fp2_sub(a0, a0, t);
  if constexpr (AT_P) {
    fp2_mul_fp(t, th, xp);
    fp2_neg(a1, t);
    fp2_mul_fp(b1, la, yp);
  } else {
    a1 = th;
    b1 = la;
  }
  // point
  fp2_sqr(C, th);
  fp2_sqr(D, la);
  fp2_mul(E, D, la);
  fp2_mul(F, T.z, C);
  fp2_mul(G, T.x, D);
  fp2_add(H, E, F);
  fp2_sub(H, H, G);
  fp2_sub(H, H, G);
  fp2_mul(T.x, la, H);
  fp2_sub(t, G, H);
  fp2_mul(t, th, t);
  fp2_mul(C, T.y, E);
  fp2_sub(T.y, t, C);
  fp2_mul(T.z, T.z, E);
}
BGV_NIS void miller_add_step(g2p_t& T, fp2_t& a0, fp2_t& a1, fp2_t& b1, const g2a& Q, const fp_t& xp,
                            const fp_t& yp) {
  miller_add_core<true>(T, a0, a1, b1, Q, xp, yp);
}

// Fixed-argument lines (BGV_LINES): the 68 lines of Q's Miller loop (63
// doublings, 5 additions), unevaluated, stored per step as (a0, a1, b1) at
// lines[(3 step + c) stride + i]; miller_line_at_p finishes one at P with
// the operations the steps above apply, so f is bit-identical.
constexpr int MILLER_STEPS = 68;
#ifndef BGV_LINES_INLINE
#define BGV_LINES_INLINE 1  // into k_lines: scratch 960 -> 496 B/lane (r04)
#endif
#if BGV_LINES_INLINE
BGV_HD
#else
BGV_NI
#endif
void miller_lines(fp2_t* lines, uint32_t stride, uint32_t i, const g2a& Q) {
  g2p_t T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp2_t a0, a1, b1;
  fp_t zero;
  fp_set_zero(zero);
  uint32_t s = 0;
  for (int b = 62; b >= 0; b--) {
    miller_dbl_core<false>(T, a0, a1, b1, zero, zero);
    lines[(size_t)(3 * s) * stride + i] = a0;
    lines[(size_t)(3 * s + 1) * stride + i] = a1;
    lines[(size_t)(3 * s + 2) * stride + i] = b1;
    s++;
    if ((BLS_X_ABS >> b) & 1ull) {
      miller_add_core<false>(T, a0, a1, b1, Q, zero, zero);
      lines[(size_t)(3 * s) * stride + i] = a0;
      lines[(size_t)(3 * s + 1) * stride + i] = a1;
      lines[(size_t)(3 * s + 2) * stride + i] = b1;
      s++;
    }
  }
}

BGV_HD void miller_line_at_p(fp2_t& a0, fp2_t& a1, fp2_t& b1, const fp2_t* lines, uint32_t stride,
                                                 uint32_t i, uint32_t s, bool add, const fp_t& xp, const fp_t& yp) {
  fp2_t t;
  a0 = lines[(size_t)(3 * s) * stride + i];
  const fp2_t c1 = lines[(size_t)(3 * s + 1) * stride + i], c2 = lines[(size_t)(3 * s + 2) * stride + i];
  if (!add) {
    fp2_mul_fp(a1, c1, xp);
    fp2_mul_fp(t, c2, yp);
    fp2_neg(b1, t);
  } else {
    fp2_mul_fp(t, c1, xp);
    fp2_neg(a1, t);
    fp2_mul_fp(b1, c2, yp);
  }
}

// f = f_{x, Q}(P) for the negative x (conjugated), P affine in G1, Q affine in G2.
// P or Q at infinity gives 1.
BGV_NI void miller_loop(fp12_t& f, const g1a& P, bool p_inf, const g2a& Q, bool q_inf) {
  fp12_one(f);
  if (p_inf || q_inf) return;
  g2p_t T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp2_t a0, a1, b1;
  bool first = true;
  for (int b = 62; b >= 0; b--) {
    if (!first) fp12_sqr(f, f);
    miller_dbl_step(T, a0, a1, b1, P.x, P.y);
    if (first) {
      // f = 1 * line
      fp12_one(f);
      f.c0.c0 = a0;
      f.c0.c1 = a1;
      f.c1.c1 = b1;
      first = false;
    } else {
      fp12_mul_line(f, f, a0, a1, b1);
    }
    if ((BLS_X_ABS >> b) & 1ull) {
      miller_add_step(T, a0, a1, b1, Q, P.x, P.y);
      fp12_mul_line(f, f, a0, a1, b1);
    }
  }
  fp12_conj(f, f);  // x < 0
}

// Two pairs with ONE shared accumulator: f = f_{x,Q1}(P1) * f_{x,Q2}(P2),
// so the Fp12 squaring of every iteration is paid once for both pairs
// (the multi-Miller loop of blst's miller_loop_n, at width 2).
BGV_NIL void miller_loop2(fp12_t& f, const g1a& P1, const g2a& Q1, const g1a& P2, const g2a& Q2) {
  g2p_t T1, T2;
  T1.x = Q1.x; T1.y = Q1.y; T1.z = fp2_one();
  T2.x = Q2.x; T2.y = Q2.y; T2.z = fp2_one();
  fp2_t a0, a1, b1;
  fp12_one(f);
  for (int b = 62; b >= 0; b--) {
    if (b != 62) fp12_sqr(f, f);
    miller_dbl_step(T1, a0, a1, b1, P1.x, P1.y);
#if BGV_MILLER_LINE2
    if (b != 62) {
      fp2_t c0, c1, d1;
      miller_dbl_step(T2, c0, c1, d1, P2.x, P2.y);
      fp12_mul_line2(f, f, a0, a1, b1, c0, c1, d1);
    } else
#endif
    {
      if (b == 62) {  // f = 1 * line
        f.c0.c0 = a0;
        f.c0.c1 = a1;
        f.c1.c1 = b1;
      } else {
        fp12_mul_line(f, f, a0, a1, b1);
      }
      miller_dbl_step(T2, a0, a1, b1, P2.x, P2.y);
      fp12_mul_line(f, f, a0, a1, b1);
    }
    if ((BLS_X_ABS >> b) & 1ull) {
      miller_add_step(T1, a0, a1, b1, Q1, P1.x, P1.y);
#if BGV_MILLER_LINE2
      fp2_t c0, c1, d1;
      miller_add_step(T2, c0, c1, d1, Q2, P2.x, P2.y);
      fp12_mul_line2(f, f, a0, a1, b1, c0, c1, d1);
#else
      fp12_mul_line(f, f, a0, a1, b1);
      miller_add_step(T2, a0, a1, b1, Q2, P2.x, P2.y);
      fp12_mul_line(f, f, a0, a1, b1);
#endif
    }
  }
  fp12_conj(f, f);  // x < 0
}

// miller_loop2 (two = true) / miller_loop over precomputed lines of sets i1, i2
BGV_NIL void miller_loop_lines(fp12_t& f, const fp2_t* lines, uint32_t stride, const g1a& P1, uint32_t i1,
                               const g1a& P2, uint32_t i2, bool two) {
  fp2_t a0, a1, b1;
  fp12_one(f);
  uint32_t s = 0;
  for (int b = 62; b >= 0; b--) {
    if (b != 62) fp12_sqr(f, f);
    miller_line_at_p(a0, a1, b1, lines, stride, i1, s, false, P1.x, P1.y);
#if BGV_MILLER_LINE2
    if (two && b != 62) {
      fp2_t c0, c1, d1;
      miller_line_at_p(c0, c1, d1, lines, stride, i2, s, false, P2.x, P2.y);
      fp12_mul_line2(f, f, a0, a1, b1, c0, c1, d1);
    } else
#endif
    {
      if (b == 62) {  // f = 1 * line
        f.c0.c0 = a0;
        f.c0.c1 = a1;
        f.c1.c1 = b1;
      } else {
        fp12_mul_line(f, f, a0, a1, b1);
      }
      if (two) {
        miller_line_at_p(a0, a1, b1, lines, stride, i2, s, false, P2.x, P2.y);
        fp12_mul_line(f, f, a0, a1, b1);
      }
    }
    s++;
    if ((BLS_X_ABS >> b) & 1ull) {
      miller_line_at_p(a0, a1, b1, lines, stride, i1, s, true, P1.x, P1.y);
#if BGV_MILLER_LINE2
      if (two) {
        fp2_t c0, c1, d1;
        miller_line_at_p(c0, c1, d1, lines, stride, i2, s, true, P2.x, P2.y);
        fp12_mul_line2(f, f, a0, a1, b1, c0, c1, d1);
      } else
#endif
      {
        fp12_mul_line(f, f, a0, a1, b1);
        if (two) {
          miller_line_at_p(a0, a1, b1, lines, stride, i2, s, true, P2.x, P2.y);
          fp12_mul_line(f, f, a0, a1, b1);
        }
      }
      s++;
    }
  }
  fp12_conj(f, f);  // x < 0
}

// a line forced to 1 (a0 = 1, a1 = b1 = 0) where `live` is false: the dummy
// pairs of an item with fewer than four sets leave f unchanged, and every lane
// issues the same products (no divergent tail for a job's last item)
BGV_HD void miller_line_keep(fp2_t& a0, fp2_t& a1, fp2_t& b1, bool live) {
  const fp2_t one = fp2_one(), zero = fp2_zero();
  fp2_select(a0, live, a0, one);
  fp2_select(a1, live, a1, zero);
  fp2_select(b1, live, b1, zero);
}

// Four pairs with ONE shared accumulator over precomputed lines (pairs_per_item
// = 4): f = prod_k f_{x,Q_k}(P_k) for the cnt (1..4) live pairs at sets
// i[0..3] (a dead pair's index is any live set, its line is forced to 1).  Per
// doubling step one Fp12 squaring serves four pairs instead of two, and the
// lines enter two at a time (fp12_mul_line2): 12 + 2 x 23 Fp2 products per
// step against 2 x (12 + 23) for two two-pair items, ~570 fewer Fp products
// per set at C4.  The product is the same element of Fp12 as the two-pair
// loops' (each line's factor is exact), and its final exponentiation is what
// the stage tests compare.
BGV_NIL void miller_loop_lines4(fp12_t& f, const fp2_t* lines, uint32_t stride, const g1a& P0, const g1a& P1,
                                const g1a& P2, const g1a& P3, uint32_t i0, uint32_t i1, uint32_t i2, uint32_t i3,
                                uint32_t cnt) {
  fp2_t a0, a1, b1, c0, c1, d1;
  fp12_one(f);
  uint32_t s = 0;
  for (int b = 62; b >= 0; b--) {
    const bool add = ((BLS_X_ABS >> b) & 1ull) != 0;
    for (int k = 0; k < (add ? 2 : 1); k++) {
      const bool ad = k == 1;
      if (b != 62 && !ad) fp12_sqr(f, f);
      miller_line_at_p(a0, a1, b1, lines, stride, i0, s, ad, P0.x, P0.y);
      miller_line_at_p(c0, c1, d1, lines, stride, i1, s, ad, P1.x, P1.y);
      miller_line_keep(c0, c1, d1, cnt > 1);
      fp12_mul_line2(f, f, a0, a1, b1, c0, c1, d1);
      miller_line_at_p(a0, a1, b1, lines, stride, i2, s, ad, P2.x, P2.y);
      miller_line_keep(a0, a1, b1, cnt > 2);
      miller_line_at_p(c0, c1, d1, lines, stride, i3, s, ad, P3.x, P3.y);
      miller_line_keep(c0, c1, d1, cnt > 3);
      fp12_mul_line2(f, f, a0, a1, b1, c0, c1, d1);
      s++;
    }
  }
  fp12_conj(f, f);  // x < 0
}

}  // namespace bgv
