// Two-lane Miller loop ("duo"): lanes 2k and 2k+1 of a wave share one pair.
//
// Lane h owns the half f_h of the accumulator f = f_0 + f_1 w (Fp12 = Fp6[w])
// in registers, and both lanes hold the same copy of T.  Every step is split
// into two equal streams of Fp2 products that the two lanes run in SIMT
// lockstep (the SAME instructions on lane-selected operands), so a pair's
// dependent chain is ~19 Fp2 products per iteration instead of the one-lane
// loop's ~35, with ~5% more products in total (the 6-lane layout of
// miller_coop.h spends ~50% more):
//   S  f^2: lane 1 t = f_0 f_1, lane 0 s = (f_0 + f_1)(f_0 + v f_1)   6 + 6
//      (complex squaring: f_0' = s - t - v t, f_1' = 2 t)
//   D  doubling step (pairing.h miller_dbl_core, same formulas), two rounds:
//      lane 0 XY, Y^2 | lane 1 Z^2, (Y+Z)^2, both X^2;  then
//      lane 0 A (B - F), E^2, 3X^2 xP | lane 1 B H, G^2, H yP        3 + 3
//   L  f * (a0 + a1 w^2 + b1 w^3): lane 0 P1 = f_0 (a0, a1, 0), lane 1
//      P3 = (f_0 + f_1)(a0, a1 + b1, 0); P2 = f_1 (b1 v) split over both
//      (f_0' = P1 + v P2, f_1' = P3 - P1 - P2)                         7 + 7
// The 5 addition steps run redundantly on both lanes.  Values cross between
// the two lanes through a per-pair LDS slot; a wave's LDS accesses execute in
// issue order, so only the compiler must keep them in order (coop_wave_sync).
// Every field value is fully reduced, so f is bit-identical to miller_loop().
#pragma once
#include "miller_coop.h"

namespace bgv {

struct duo_x_t {
  fp6_t fx[2];  // published halves of f / the line products P1, P3
  fp2_t dx[6];  // doubling-step products / parts of P2
};

__device__ __forceinline__ void duo_sel6(fp6_t& r, bool c, const fp6_t& a, const fp6_t& b) {
  fp2_select(r.c0, c, a.c0, b.c0);
  fp2_select(r.c1, c, a.c1, b.c1);
  fp2_select(r.c2, c, a.c2, b.c2);
}
__device__ __forceinline__ fp2_t duo_sel2(bool c, const fp2_t& a, const fp2_t& b) {
  fp2_t r;
  fp2_select(r, c, a, b);
  return r;
}

// both halves of f: (f0, f1) from this lane's fh and the other lane's
__device__ __forceinline__ void duo_halves(fp6_t& f0, fp6_t& f1, const fp6_t& fh, uint32_t h, duo_x_t& X) {
  X.fx[h] = fh;
  coop_wave_sync();
  const fp6_t fo = X.fx[h ^ 1u];
  coop_wave_sync();  // both halves read before the slots are reused
  duo_sel6(f0, h != 0, fo, fh);
  duo_sel6(f1, h != 0, fh, fo);
}

// f <- f^2
__device__ __forceinline__ void duo_sqr(fp6_t& fh, uint32_t h, duo_x_t& X) {
  fp6_t f0, f1, s, t, a, b;
  duo_halves(f0, f1, fh, h, X);
  fp6_add(s, f0, f1);
  fp6_mul_v(t, f1);
  fp6_add(t, f0, t);
  duo_sel6(a, h != 0, f0, s);  // lane 1: f0 f1, lane 0: (f0 + f1)(f0 + v f1)
  duo_sel6(b, h != 0, f1, t);
  fp6_t r;
  fp6_mul(r, a, b);
  if (h) X.fx[1] = r;
  coop_wave_sync();
  const fp6_t tt = X.fx[1];  // t = f0 f1
  coop_wave_sync();
  fp6_t c0, c1, vt;
  fp6_add(c1, tt, tt);
  fp6_mul_v(vt, tt);
  fp6_sub(c0, r, tt);
  fp6_sub(c0, c0, vt);
  duo_sel6(fh, h != 0, c1, c0);
}

// doubling step (pairing.h miller_dbl_core<true>): T <- 2T, line at P
__device__ __forceinline__ void duo_dbl(g2p_t& T, fp2_t& a0, fp2_t& a1, fp2_t& b1, const fp_t& xp, const fp_t& yp,
                                        uint32_t h, duo_x_t& X) {
  const bool hi = h != 0;
  fp2_t yz, m1, m2, x2;
  fp2_add(yz, T.y, T.z);
  {
    const fp2_t p = duo_sel2(hi, T.z, T.x), q = duo_sel2(hi, T.z, T.y), r = duo_sel2(hi, yz, T.y);
    fp2_mul(m1, p, q);  // lane 0 XY | lane 1 Z^2
    fp2_sqr(m2, r);     // lane 0 Y^2 | lane 1 (Y+Z)^2
    fp2_sqr(x2, T.x);   // both X^2
  }
  X.dx[2 * h] = m1;
  X.dx[2 * h + 1] = m2;
  coop_wave_sync();
  const fp2_t xy = X.dx[0], B = X.dx[1], C = X.dx[2], yz2 = X.dx[3];
  coop_wave_sync();
  fp2_t A, E, F, H, t;
  A = xy;
  fp_half(A.c0, A.c0);
  fp_half(A.c1, A.c1);  // XY/2
  fp2_mul_3b(E, C);     // 3b' Z^2
  fp2_mul3(F, E);
  fp2_add(H, B, C);
  fp2_sub(H, yz2, H);   // 2YZ
  fp2_sub(a0, E, B);
  fp2_t bf, g, x3;
  fp2_sub(bf, B, F);
  fp2_add(g, B, F);
  fp_half(g.c0, g.c0);
  fp_half(g.c1, g.c1);  // (B + F)/2
  fp2_mul3(x3, x2);     // 3X^2
  {
    const fp2_t p = duo_sel2(hi, B, A), q = duo_sel2(hi, H, bf), r = duo_sel2(hi, g, E), s = duo_sel2(hi, H, x3);
    const fp_t& u = hi ? yp : xp;
    fp2_mul(m1, p, q);      // lane 0 X' = A (B - F) | lane 1 Z' = B H
    fp2_sqr(m2, r);         // lane 0 E^2 | lane 1 G^2
    fp2_mul_fp(t, s, u);    // lane 0 a1 = 3X^2 xP | lane 1 H yP
  }
  X.dx[3 * h] = m1;
  X.dx[3 * h + 1] = m2;
  X.dx[3 * h + 2] = t;
  coop_wave_sync();
  const fp2_t nx = X.dx[0], e2 = X.dx[1], ta1 = X.dx[2], nz = X.dx[3], g2 = X.dx[4], hy = X.dx[5];
  coop_wave_sync();
  a1 = ta1;
  fp2_neg(b1, hy);
  fp2_mul3(t, e2);
  T.x = nx;
  fp2_sub(T.y, g2, t);  // G^2 - 3E^2
  T.z = nz;
}

// f <- f * (a0 + a1 w^2 + b1 w^3)
__device__ __forceinline__ void duo_line(fp6_t& fh, const fp2_t& a0, const fp2_t& a1, const fp2_t& b1, uint32_t h,
                                         duo_x_t& X) {
  const bool hi = h != 0;
  fp6_t f0, f1, s, a, r;
  duo_halves(f0, f1, fh, h, X);
  fp6_add(s, f0, f1);
  duo_sel6(a, hi, s, f0);
  fp2_t c, ab;
  fp2_add(ab, a1, b1);
  c = duo_sel2(hi, ab, a1);
  fp6_mul_01(r, a, a0, c);  // lane 0 P1 = f0 (a0, a1, 0) | lane 1 P3 = (f0 + f1)(a0, a1 + b1, 0)
  fp2_t u, vv;
  {
    const fp2_t p = duo_sel2(hi, f1.c1, f1.c2);
    fp2_mul(u, p, b1);        // lane 0 f1.c2 b1 (P2.c0 / xi) | lane 1 f1.c1 b1 (P2.c2)
    fp2_mul(vv, f1.c0, b1);   // both P2.c1
  }
  X.fx[h] = r;
  X.dx[h] = u;
  coop_wave_sync();
  const fp6_t p1 = X.fx[0], p3 = X.fx[1];
  const fp2_t u0 = X.dx[0], u1 = X.dx[1];
  coop_wave_sync();
  fp6_t p2, o0, o1;
  fp2_mul_xi(p2.c0, u0);
  p2.c1 = vv;
  p2.c2 = u1;
  fp6_t vp2;
  fp6_mul_v(vp2, p2);
  fp6_add(o0, p1, vp2);
  fp6_sub(o1, p3, p1);
  fp6_sub(o1, o1, p2);
  duo_sel6(fh, hi, o1, o0);
}

// the pair (P, Q) on lanes (2k, 2k+1): fh = this lane's half of f_{x,Q}(P)
// for the negative x (conjugated)
__device__ void duo_miller(fp6_t& fh, const g1a& P, const g2a& Q, uint32_t h, duo_x_t& X) {
  g2p_t T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp2_t a0, a1, b1;
  for (int bit = 62; bit >= 0; bit--) {
    if (bit != 62) duo_sqr(fh, h, X);
    duo_dbl(T, a0, a1, b1, P.x, P.y, h, X);
    if (bit == 62) {  // f = 1 * line: f0 = (a0, a1, 0), f1 = (0, b1, 0)
      fp6_t l0, l1;
      l0.c0 = a0; l0.c1 = a1; l0.c2 = fp2_zero();
      l1.c0 = fp2_zero(); l1.c1 = b1; l1.c2 = fp2_zero();
      duo_sel6(fh, h != 0, l1, l0);
    } else {
      duo_line(fh, a0, a1, b1, h, X);
    }
    if ((BLS_X_ABS >> bit) & 1ull) {
      miller_add_core<true>(T, a0, a1, b1, Q, P.x, P.y);  // both lanes, same values
      duo_line(fh, a0, a1, b1, h, X);
    }
  }
  if (h) fp6_neg(fh, fh);  // x < 0: conjugate (negate f1)
}

}  // namespace bgv
