// Four-lane Miller loop ("quad"): lanes 4k .. 4k+3 of a wave share one pair.
//
// Lane rho = 2h + s.  Half h owns f_h of f = f_0 + f_1 w (Fp12 = Fp6[w]) in
// registers, as in the two-lane loop (miller_duo.h); sub-lane s splits every
// Fp6-level product of that half, and the doubling step's products go one per
// lane.  Every lane issues the SAME sequence of product calls per iteration
// (4 + 1 + 1 + 4 Fp2-sized calls, 29 Fp products against the one-lane loop's
// 95) on lane-selected operands:
//   S  f^2 = (u - t - v t) + 2 t w, u = (f0 + f1)(f0 + v f1), t = f0 f1:
//      the six Karatsuba products of u on half 0, of t on half 1, three per
//      sub-lane (s = 0: a_k b_k, s = 1: (a_i + a_j)(b_i + b_j));
//      in the same rounds the doubling step's XY, Y^2, Z^2, (Y + Z)^2
//   D  A (B - F), E^2, G^2, B H one per lane; then 3X^2 xP, H yP
//      (X^2 of T comes from the previous line round's spare slot)
//   L  f * (a0 + a1 v + b1 v w): P1 = F0 (a0 + a1 v) on half 0 with
//      P2 = F1 b1 v, P3 = (F0 + F1)(a0 + (a1 + b1) v) on half 1, plus X'^2
// Operands come from per-pair LDS slots through lane-dependent addresses (a
// free selection); a wave's LDS accesses execute in issue order, so only the
// compiler must keep them in order (coop_wave_sync).  The five addition steps
// spread their products over the lanes too (quad_add).  Every field value is fully reduced, so f is
// bit-identical to miller_loop().
#pragma once
#include "miller_coop.h"

namespace bgv {

struct quad_x_t {
  fp2_t F[6];   // published f halves (F[3h + k]); in the S recombination the Fp6 values u / t; in L, F0 / F1
  fp2_t R[16];  // product exchange: R[4 rho + round]
  fp2_t L[4];   // line a0, a1, b1, a1 + b1
};                // 26 Fp2 = 2,496 B per pair (+ one zero slot per block): 4 waves (64 pairs) per CU

__device__ __forceinline__ fp2_t q_sel4(uint32_t r, const fp2_t& a, const fp2_t& b, const fp2_t& c, const fp2_t& d) {
  fp2_t x, y, z;
  fp2_select(x, (r & 1u) != 0, b, a);
  fp2_select(y, (r & 1u) != 0, d, c);
  fp2_select(z, (r & 2u) != 0, y, x);
  return z;
}
__device__ __forceinline__ fp2_t q_sel2(bool c, const fp2_t& a, const fp2_t& b) {
  fp2_t r;
  fp2_select(r, c, a, b);
  return r;
}
__device__ __forceinline__ fp2_t q_lazy(const fp2_t& a, const fp2_t& b) {  // < 2p: product inputs only
  fp2_t r;
  fp_add_lazy2(r.c0, a.c0, b.c0, r.c1, a.c1, b.c1);
  return r;
}

// Karatsuba pairs of the s = 1 sub-lane: q0 = (0,1), q1 = (0,2), q2 = (1,2)
BGV_CONST uint8_t QUAD_PI[3] = {0, 0, 1};
BGV_CONST uint8_t QUAD_PJ[3] = {1, 2, 2};

// Operands that are conditionally zero are read through a lane-selected LDS
// address, the per-block zero slot zp standing for 0 (one address select
// instead of a 24-dword value select per operand; BGV_QUAD_ZSLOT 0: value select)
#ifndef BGV_QUAD_ZSLOT
#define BGV_QUAD_ZSLOT 1
#endif
#if BGV_QUAD_ZSLOT
#define QUAD_OR_ZERO(c, p) (*((c) ? (p) : zp))
#else
#define QUAD_OR_ZERO(c, p) q_sel2((c), *(p), fp2_zero())
#endif
// S-round operand X(m) of half h: f0[m] + f1[m] (h = 0, a = f0 + f1) or f0[m]
// (h = 1); 0 when `zero` (sub-lane 0's unpaired second operand)
__device__ __forceinline__ fp2_t quad_sx(const quad_x_t& X, uint32_t h, uint32_t m, const fp2_t* zp, bool zero) {
  const fp2_t f0 = QUAD_OR_ZERO(!zero, &X.F[m]);
  const fp2_t f1 = QUAD_OR_ZERO(!zero && !h, &X.F[3 + m]);
  fp2_t r;
  fp2_add(r, f0, f1);
  return r;
}
// S-round operand Y(m): f0[m] + (v f1)[m] (h = 0, b = f0 + v f1) or f1[m] (h = 1);
// (v f1) = (xi f1[2], f1[0], f1[1]); 0 when `zero`
__device__ __forceinline__ fp2_t quad_sy(const quad_x_t& X, uint32_t h, uint32_t m, const fp2_t* zp, bool zero) {
  const uint32_t i1 = h ? m : (m + 2u) % 3u;
  fp2_t g = QUAD_OR_ZERO(!zero, &X.F[3 + i1]);
  fp2_t gx;
  fp2_mul_xi(gx, g);
  g = q_sel2(!h && m == 0, gx, g);
  const fp2_t f0 = QUAD_OR_ZERO(!zero && !h, &X.F[m]);
  fp2_t r;
  fp2_add(r, f0, g);
  return r;
}

// the doubling step of T (pairing.h miller_dbl_core<true>, same formulas) over
// the four lanes, its first round folded into the caller's S rounds: d1 is
// this lane's product of that round (rho 0: XY, 1: Y^2, 2: Z^2, 3: (Y+Z)^2),
// published at X.R[4 rho + 3] before the call.  Leaves T' in T and the line
// (a0, a1, b1) in X.L[0..3] (with a1 + b1); x2 = X^2 of the old T.
__device__ __forceinline__ void quad_dbl_tail(g2p_t& T, const fp2_t& x2, const fp_t& xp, const fp_t& yp, uint32_t rho,
                                              quad_x_t& X) {
  const fp2_t xy = X.R[3], B = X.R[7], C = X.R[11], yz2 = X.R[15];
  fp2_t A, E, F, H, a0, bf, g, x3;
  A = xy;
  fp_half(A.c0, A.c0);
  fp_half(A.c1, A.c1);  // XY/2
  fp2_mul_3b(E, C);
  fp2_mul3(F, E);
  fp2_add(H, B, C);
  fp2_sub(H, yz2, H);   // 2YZ
  fp2_sub(a0, E, B);
  fp2_sub(bf, B, F);
  fp2_add(g, B, F);
  fp_half(g.c0, g.c0);
  fp_half(g.c1, g.c1);  // (B + F)/2
  fp2_mul3(x3, x2);     // 3X^2
  fp2_t m1, m2;
  {
    const fp2_t p = q_sel4(rho, A, E, g, B), q = q_sel4(rho, bf, E, g, H);
    fp2_mul(m1, p, q);  // rho 0: X' = A (B - F) | 1: E^2 | 2: G^2 | 3: Z' = B H
    const fp2_t u = q_sel2((rho & 1u) != 0, H, x3);
    const fp_t& w = (rho & 1u) ? yp : xp;
    fp2_mul_fp(m2, u, w);  // even: a1 = 3X^2 xP | odd: H yP
  }
  coop_wave_sync();  // every lane has read R[3], R[7], R[11], R[15]
  X.R[4 * rho] = m1;
  X.R[4 * rho + 1] = m2;
  coop_wave_sync();
  const fp2_t nx = X.R[0], e2 = X.R[4], g2 = X.R[8], nz = X.R[12], a1 = X.R[1], hy = X.R[5];
  fp2_t b1, t;
  fp2_neg(b1, hy);
  fp2_mul3(t, e2);
  T.x = nx;
  fp2_sub(T.y, g2, t);  // G^2 - 3E^2
  T.z = nz;
  fp2_t ab;
  fp2_add(ab, a1, b1);
  coop_wave_sync();  // R read by every lane before the line round overwrites it
  if (rho == 0) {
    X.L[0] = a0;
    X.L[1] = a1;
    X.L[2] = b1;
    X.L[3] = ab;
  }
}

// S rounds (three Karatsuba products of this half's Fp6 product per lane)
// plus the doubling step's first round; then the Fp6 recombination of u / t,
// published to X.F, and the doubling tail.  fh is this lane's half of f
// (consumed); leaves this lane's half of f^2 in fh.
__device__ __forceinline__ void quad_sqr_dbl(fp6_t& fh, g2p_t& T, const fp2_t& x2, const fp_t& xp, const fp_t& yp,
                                             uint32_t h, uint32_t s, uint32_t rho, quad_x_t& X, const fp2_t* zp) {
  if (s == 0) {
    X.F[3 * h] = fh.c0;
    X.F[3 * h + 1] = fh.c1;
    X.F[3 * h + 2] = fh.c2;
  }
  coop_wave_sync();
#pragma unroll 1
  for (uint32_t k = 0; k < 3; k++) {
    const uint32_t i = s ? QUAD_PI[k] : k, j = QUAD_PJ[k];
    const fp2_t xa = quad_sx(X, h, i, zp, false), ya = quad_sy(X, h, i, zp, false);
    const fp2_t xb = quad_sx(X, h, j, zp, s == 0), yb = quad_sy(X, h, j, zp, s == 0);
    fp2_t r;
    fp2_mul(r, q_lazy(xa, xb), q_lazy(ya, yb));
    X.R[4 * rho + k] = r;  // R is disjoint from F: no ordering hazard
  }
  {
    fp2_t yz;
    fp2_add(yz, T.y, T.z);
    const fp2_t p = q_sel4(rho, T.x, T.y, T.z, yz), q = q_sel4(rho, T.y, T.y, T.z, yz);
    fp2_t r;
    fp2_mul(r, p, q);  // rho 0: XY | 1: Y^2 | 2: Z^2 | 3: (Y + Z)^2
    X.R[4 * rho + 3] = r;
  }
  coop_wave_sync();
  // Fp6 Karatsuba recombination of this half's product (both sub-lanes)
  fp6_t c;
  {
    const uint32_t b0 = 8 * h;  // R[b0 + k]: sub-lane 0 (a_k b_k), R[b0 + 4 + k]: sub-lane 1 (pairs)
    const fp2_t p0 = X.R[b0], p1 = X.R[b0 + 1], p2 = X.R[b0 + 2];
    const fp2_t q01 = X.R[b0 + 4], q02 = X.R[b0 + 5], q12 = X.R[b0 + 6];
    fp2_t t;
    fp2_sub(t, q12, p1);
    fp2_sub(t, t, p2);
    fp2_mul_xi(t, t);
    fp2_add(c.c0, p0, t);  // p0 + xi (q12 - p1 - p2)
    fp2_mul_xi(t, p2);
    fp2_sub(c.c1, q01, p0);
    fp2_sub(c.c1, c.c1, p1);
    fp2_add(c.c1, c.c1, t);  // q01 - p0 - p1 + xi p2
    fp2_sub(c.c2, q02, p0);
    fp2_sub(c.c2, c.c2, p2);
    fp2_add(c.c2, c.c2, p1);  // q02 - p0 - p2 + p1
  }
  // u (half 0) and t (half 1) cross through X.F (its f values are consumed)
  coop_wave_sync();
  if (s == 0) {
    X.F[3 * h] = c.c0;
    X.F[3 * h + 1] = c.c1;
    X.F[3 * h + 2] = c.c2;
  }
  quad_dbl_tail(T, x2, xp, yp, rho, X);
  coop_wave_sync();
  fp6_t o;
  o.c0 = X.F[3 * (h ^ 1u)];
  o.c1 = X.F[3 * (h ^ 1u) + 1];
  o.c2 = X.F[3 * (h ^ 1u) + 2];
  // half 0 holds u (c) and reads t (o): f0 = u - t - v t; half 1 holds t: f1 = 2 t.
  // Both formulas run on every lane on (c, o) and the lane keeps its own.
  fp6_t f0, f1, vt;
  fp6_mul_v(vt, o);
  fp6_sub(f0, c, o);
  fp6_sub(f0, f0, vt);  // u - t - v t (half 0)
  fp6_add(f1, c, c);    // 2 t (half 1)
  duo_sel6(fh, h != 0, f1, f0);
}

// line-round operand of lane rho, round r: (F0[i] w0 + F1[i] w1 (+ the same
// at j when paired)) * (L[li] (+ L[lj]))
struct quad_op {
  uint8_t i, j, w0, w1, pair, li, lj, lpair;
};
BGV_CONST quad_op QUAD_L[4][4] = {
    {{0, 0, 1, 0, 0, 0, 0, 0}, {1, 0, 1, 0, 0, 1, 0, 0}, {2, 0, 1, 0, 0, 1, 0, 0}, {2, 0, 0, 1, 0, 2, 0, 0}},
    {{0, 1, 1, 0, 1, 0, 1, 1}, {2, 0, 1, 0, 0, 0, 0, 0}, {0, 0, 0, 1, 0, 2, 0, 0}, {1, 0, 0, 1, 0, 2, 0, 0}},
    {{0, 0, 1, 1, 0, 0, 0, 0}, {1, 0, 1, 1, 0, 3, 0, 0}, {2, 0, 1, 1, 0, 3, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}},
    {{0, 1, 1, 1, 1, 0, 3, 1}, {2, 0, 1, 1, 0, 0, 0, 0}, {0, 0, 1, 0, 0, 0, 0, 0}, {0, 0, 1, 0, 0, 0, 0, 0}},
};

// f <- f * (a0 + a1 v + b1 v w) with the line in X.L; this lane's half of f
// in fh.  The spare slot of lane 2 squares T.x: x2 = X^2 of the new T.
__device__ __forceinline__ void quad_line(fp6_t& fh, fp2_t& x2, const g2p_t& T, uint32_t h, uint32_t s, uint32_t rho,
                                          quad_x_t& X, const fp2_t* zp) {
  // publish F0 / F1 (X.F is free: every lane has read the u / t values)
  coop_wave_sync();
  if (s == 0) {
    X.F[3 * h] = fh.c0;
    X.F[3 * h + 1] = fh.c1;
    X.F[3 * h + 2] = fh.c2;
  }
  coop_wave_sync();
  // round r, lane rho: product A * B with
  //   rho 0: m0 = F0[0] a0, m1 = F0[1] a1, m2 = F0[2] a1, n0 = F1[2] b1
  //   rho 1: m3 = (F0[0] + F0[1])(a0 + a1), m4 = F0[2] a0, n1 = F1[0] b1, n2 = F1[1] b1
  //   rho 2: k0 = S[0] a0, k1 = S[1] a', k2 = S[2] a', X^2
  //   rho 3: k3 = (S[0] + S[1])(a0 + a'), k4 = S[2] a0, -, -
  // (S = F0 + F1, a' = a1 + b1); an operand is F0[i] w0 + F1[i] w1 (+ the same
  // at j when paired) against L[li] (+ L[lj])
#pragma unroll 1
  for (uint32_t r = 0; r < 4; r++) {
    const quad_op e = QUAD_L[rho][r];
    fp2_t a, b;
    {
      const fp2_t x0 = QUAD_OR_ZERO(e.w0 != 0, &X.F[e.i]), x1 = QUAD_OR_ZERO(e.w1 != 0, &X.F[3 + e.i]);
      const fp2_t y0 = QUAD_OR_ZERO(e.w0 && e.pair, &X.F[e.j]), y1 = QUAD_OR_ZERO(e.w1 && e.pair, &X.F[3 + e.j]);
      fp2_t ai, aj;
      fp2_add(ai, x0, x1);
      fp2_add(aj, y0, y1);
      a = q_lazy(ai, aj);
      const fp2_t l0 = X.L[e.li], l1 = QUAD_OR_ZERO(e.lpair != 0, &X.L[e.lj]);
      b = q_lazy(l0, l1);
    }
    // rho 2, round 3: X^2 of the new T (for the next doubling step's 3X^2 xP)
    const bool sq = rho == 2 && r == 3;
    a = q_sel2(sq, T.x, a);
    b = q_sel2(sq, T.x, b);
    fp2_t p;
    fp2_mul(p, a, b);
    X.R[4 * rho + r] = p;
  }
  coop_wave_sync();
  x2 = X.R[11];
  // f0'' = P1 + v P2 = (m0 + xi m2 + xi n2, m3 - m0 - m1 + xi n0, m4 + m1 + n1)
  // f1'' = P3 - P1 - P2, P3 = (k0 + xi k2, k3 - k0 - k1, k4 + k1), P2 = (xi n0, n1, n2)
  const fp2_t m0 = X.R[0], m1 = X.R[1], m2 = X.R[2], n0 = X.R[3];
  const fp2_t m3 = X.R[4], m4 = X.R[5], n1 = X.R[6], n2 = X.R[7];
  fp6_t p1, v, o0, o1;
  fp2_mul_xi(p1.c0, m2);
  fp2_add(p1.c0, p1.c0, m0);
  fp2_sub(p1.c1, m3, m0);
  fp2_sub(p1.c1, p1.c1, m1);
  fp2_add(p1.c2, m4, m1);
  // v = P2 (half 1) or v P2 (half 0): v P2 = (xi n2, xi n0, n1)
  {
    fp2_t xn0, xn2;
    fp2_mul_xi(xn0, n0);
    fp2_mul_xi(xn2, n2);
    v.c0 = q_sel2(h != 0, xn0, xn2);
    v.c1 = q_sel2(h != 0, n1, xn0);
    v.c2 = q_sel2(h != 0, n2, n1);
  }
  fp6_add(o0, p1, v);
  {
    const fp2_t k0 = X.R[8], k1 = X.R[9], k2 = X.R[10], k3 = X.R[12], k4 = X.R[13];
    fp6_t p3;
    fp2_mul_xi(p3.c0, k2);
    fp2_add(p3.c0, p3.c0, k0);
    fp2_sub(p3.c1, k3, k0);
    fp2_sub(p3.c1, p3.c1, k1);
    fp2_add(p3.c2, k4, k1);
    fp6_sub(o1, p3, o0);  // P3 - (P1 + P2)
  }
  duo_sel6(fh, h != 0, o1, o0);
}

// one exchange round: every lane publishes r at slot rho, then reads all four
__device__ __forceinline__ void quad_round(fp2_t out[4], const fp2_t& r, uint32_t rho, quad_x_t& X) {
  coop_wave_sync();  // earlier reads of these slots are done
  X.R[rho] = r;
  coop_wave_sync();
  out[0] = X.R[0];
  out[1] = X.R[1];
  out[2] = X.R[2];
  out[3] = X.R[3];
}

// the addition step (pairing.h miller_add_core<true>, same formulas and
// values) with its products spread over the four lanes: 3 + 3 + 3 + 2 + 3 Fp
// products of chain instead of ~37 on every lane.  Leaves T + Q in T and the
// line (a0, a1, b1, a1 + b1) in X.L.
__device__ __forceinline__ void quad_add(g2p_t& T, const g2a& Q, const fp_t& xp, const fp_t& yp, uint32_t rho,
                                         quad_x_t& X) {
  fp2_t o[4], r;
  // R1: yQ Z | xQ Z
  fp2_mul(r, q_sel2((rho & 1u) != 0, Q.x, Q.y), T.z);
  quad_round(o, r, rho, X);
  fp2_t th, la;
  fp2_sub(th, T.y, o[0]);  // theta = Y - yQ Z
  fp2_sub(la, T.x, o[1]);  // lambda = X - xQ Z
  // R2: th xQ | la yQ | C = th^2 | D = la^2
  fp2_mul(r, q_sel4(rho, th, la, th, la), q_sel4(rho, Q.x, Q.y, th, la));
  quad_round(o, r, rho, X);
  fp2_t a0, C, D;
  fp2_sub(a0, o[0], o[1]);
  C = o[2];
  D = o[3];
  // R3: E = D la | F = Z C | G = X D
  fp2_mul(r, q_sel4(rho, D, T.z, T.x, D), q_sel4(rho, la, C, D, la));
  quad_round(o, r, rho, X);
  const fp2_t E = o[0], F = o[1], G = o[2];
  // R3b: th xP | la yP
  fp2_mul_fp(r, q_sel2((rho & 1u) != 0, la, th), (rho & 1u) ? yp : xp);
  quad_round(o, r, rho, X);
  fp2_t a1, b1, H, gh;
  fp2_neg(a1, o[0]);
  b1 = o[1];
  fp2_add(H, E, F);
  fp2_sub(H, H, G);
  fp2_sub(H, H, G);
  fp2_sub(gh, G, H);
  // R4: X' = la H | th (G - H) | Y E | Z' = Z E
  fp2_mul(r, q_sel4(rho, la, th, T.y, T.z), q_sel4(rho, H, gh, E, E));
  quad_round(o, r, rho, X);
  T.x = o[0];
  fp2_sub(T.y, o[1], o[2]);
  T.z = o[3];
  fp2_t ab;
  fp2_add(ab, a1, b1);
  coop_wave_sync();
  if (rho == 0) {
    X.L[0] = a0;
    X.L[1] = a1;
    X.L[2] = b1;
    X.L[3] = ab;
  }
}

// the pair (P, Q) on lanes 4k .. 4k+3: fh = this lane's half of f_{x,Q}(P)
// for the negative x (conjugated)
__device__ void quad_miller(fp6_t& fh, const g1a& P, const g2a& Q, uint32_t h, uint32_t s, quad_x_t& X, const fp2_t* zp) {
  const uint32_t rho = 2 * h + s;
  g2p_t T;
  T.x = Q.x;
  T.y = Q.y;
  T.z = fp2_one();
  fp2_t x2;
  fp2_sqr(x2, T.x);
  fp6_one(fh);
  for (int bit = 62; bit >= 0; bit--) {
    if (bit == 62) {
      // f = 1: only the doubling step (its first round, then the tail)
      fp2_t yz;
      fp2_add(yz, T.y, T.z);
      const fp2_t p = q_sel4(rho, T.x, T.y, T.z, yz), q = q_sel4(rho, T.y, T.y, T.z, yz);
      fp2_t r;
      fp2_mul(r, p, q);
      coop_wave_sync();
      X.R[4 * rho + 3] = r;
      coop_wave_sync();
      quad_dbl_tail(T, x2, P.x, P.y, rho, X);
      coop_wave_sync();
      // f = line: f0 = (a0, a1, 0), f1 = (0, b1, 0)
      fp6_t l0, l1;
      l0.c0 = X.L[0]; l0.c1 = X.L[1]; l0.c2 = fp2_zero();
      l1.c0 = fp2_zero(); l1.c1 = X.L[2]; l1.c2 = fp2_zero();
      duo_sel6(fh, h != 0, l1, l0);
      fp2_sqr(x2, T.x);
    } else {
      quad_sqr_dbl(fh, T, x2, P.x, P.y, h, s, rho, X, zp);
      quad_line(fh, x2, T, h, s, rho, X, zp);
    }
    if ((BLS_X_ABS >> bit) & 1ull) {
      quad_add(T, Q, P.x, P.y, rho, X);
      quad_line(fh, x2, T, h, s, rho, X, zp);
    }
  }
  if (h) fp6_neg(fh, fh);  // x < 0: conjugate (negate f1)
}

}  // namespace bgv
