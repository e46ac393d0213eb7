// Two-pair Miller loop in Karatsuba views (mid-size latency mode).
//
// A group of 3 S lanes (S product slots x three views, kv_g2.h) runs the
// multi-Miller loop of TWO pairs with ONE shared Fp12 accumulator, the loop
// of pairing.h miller_loop2 with fp12_mul_line2: per iteration
//   f <- f^2 * (l1 l2),  l_k the tangent (or chord) lines of T_k at P_k.
// Lane (s, q) holds view q (c0, c1 or c0 + c1) of every Fp2 value: the six
// coefficients of f, both points T_k, the lines.  Additions are one Fp
// operation per lane; every Fp2 product is one Fp product per view, the
// products of a round are dealt to the slots (product j on slot j mod S), and
// after one LDS exchange the owner lanes combine the three sub-products of
// their products into views, in place (a xi-multiplied view for products
// marked so, and products by an Fp value, x_P or y_P, are view-local).  A
// second read hands every lane the views it needs.  Multiplications by xi of
// sums of products go through one batched exchange (v0 - v1, v2, 2 v0).
//
// Per iteration and lane (S = 3): 4 (f^2: two Fp6 Karatsuba products) + 4
// (tangent step, both pairs) + 4 (tangent tails) + 2 (l1 l2) + 6 (f^2 times
// l1 l2) = 20 Fp products, against 29 for the four-lane one-pair loop
// (miller_quad.h): the squaring of f is shared by the two pairs.  Every value
// is a canonical residue, so f equals miller_loop2's.
#pragma once
#include "kv_g2.h"

namespace bgv {

constexpr int MKV_NP = 17;  // products of the largest round (f^2 times l1 l2)
constexpr int MKV_NX = 8;   // values of the largest xi batch

struct mkv_scratch {
  alignas(16) fp_t P[MKV_NP][3];  // sub-products, then (in place) views: P[j][q]
  alignas(16) fp_t X[MKV_NX][3];  // xi exchange
  alignas(16) fp_t Z;             // zero
};

template <int S>
struct mkv_grp {
  mkv_scratch* sc;
  uint32_t s, q;
};

// combination slots of view q of product j's output (4-slot form (A + B) - (C + D), 3 = zero):
//   plain: q0 (0, Z, 1, Z)  q1 (2, Z, 0, 1)  q2 (2, Z, 1, 1)          v = P0 - P1 | P2 - P0 - P1 | P2 - 2 P1
//   xi   : q0 (0, 0, 2, Z)  q1 (2, Z, 1, 1)  q2 (0, 0, 1, 1)          v = 2 P0 - P2 | P2 - 2 P1 | 2 P0 - 2 P1
__device__ __forceinline__ void mkv_slots(uint32_t q, bool xi, uint32_t& ia, uint32_t& ib, uint32_t& ic,
                                          uint32_t& id) {
  if (!xi) {
    ia = q == 0 ? 0u : 2u;
    ib = 3u;
    ic = q == 1 ? 0u : 1u;
    id = q == 0 ? 3u : 1u;
  } else {
    ia = q == 1 ? 2u : 0u;
    ib = q == 1 ? 3u : 0u;
    ic = q == 0 ? 2u : 1u;
    id = q == 0 ? 3u : 1u;
  }
}

__device__ __forceinline__ const BGV_LDS fp_t* mkv_slot(const BGV_LDS mkv_scratch* L, uint32_t j, uint32_t i) {
  return i == 3u ? &L->Z : &L->P[j][i];
}

// One round of N Fp2 products: op(j, a, b) gives the views of product j's
// operands (j compile-time after unrolling); LOCAL bit j: a product by an Fp
// value (view-local, no combination); XI bit j: the output is xi times the
// product.  Afterwards mkv_get(g, j) is this lane's view of output j.
template <int S, int N, uint32_t LOCAL, uint32_t XI, class Op>
__device__ __forceinline__ void mkv_round(const mkv_grp<S>& g, Op op) {
  BGV_LDS mkv_scratch* L = (BGV_LDS mkv_scratch*)g.sc;
  constexpr int K = (N + S - 1) / S;
#pragma unroll
  for (int k = 0; k < K; k++) {
    fp_t a, b;
#pragma unroll
    for (int t = 0; t < S; t++) {
      const int j = k * S + t;
      if (j < N) {
        fp_t x, y;
        op(j, x, y);
        if (t == 0) {
          a = x;
          b = y;
        } else {
          fp_select(a, g.s == (uint32_t)t, x, a);
          fp_select(b, g.s == (uint32_t)t, y, b);
        }
      }
    }
    fp_t r;
    fp_mul(r, a, b);
    const int j = k * S + (int)g.s;
    if (j < N) lds_put(&L->P[j][g.q], r);
  }
  coop_wave_sync();
  // owner lanes: view q of their products, in place (all reads precede the writes)
  fp_t o[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t j = (uint32_t)(k * S) + g.s;
    const uint32_t jj = j < (uint32_t)N ? j : 0u;
    const bool xi = (XI >> jj) & 1u;
    uint32_t ia, ib, ic, id;
    mkv_slots(g.q, xi, ia, ib, ic, id);
    const fp_t A = lds_get(mkv_slot(L, jj, ia)), B = lds_get(mkv_slot(L, jj, ib)), C = lds_get(mkv_slot(L, jj, ic)),
               D = lds_get(mkv_slot(L, jj, id));
    fp_t u, v;
    fp_add2(u, A, B, v, C, D);
    fp_sub(o[k], u, v);
    if ((LOCAL >> jj) & 1u) o[k] = lds_get(&L->P[jj][g.q]);
  }
  coop_wave_sync();
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t j = (uint32_t)(k * S) + g.s;
    if (j < (uint32_t)N) lds_put(&L->P[j][g.q], o[k]);
  }
  coop_wave_sync();
}

template <int S>
__device__ __forceinline__ fp_t mkv_get(const mkv_grp<S>& g, int j) {
  const BGV_LDS mkv_scratch* L = (const BGV_LDS mkv_scratch*)g.sc;
  return lds_get(&L->P[j][g.q]);
}

// xi x_k for k < n in one exchange: views (v0 - v1, v2, 2 v0) as (A + B) - C:
//   q0 (0, Z, 1)  q1 (2, Z, Z)  q2 (0, 0, Z)
template <int S, int N>
__device__ __forceinline__ void mkv_xi(const mkv_grp<S>& g, fp_t (&x)[N]) {
  BGV_LDS mkv_scratch* L = (BGV_LDS mkv_scratch*)g.sc;
  if (g.s == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) lds_put(&L->X[k][g.q], x[k]);
  }
  coop_wave_sync();
  const uint32_t ia = g.q == 1 ? 2u : 0u, ib = g.q == 2 ? 0u : 3u, ic = g.q == 0 ? 1u : 3u;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const fp_t A = lds_get(ia == 3u ? &L->Z : &L->X[k][ia]), B = lds_get(ib == 3u ? &L->Z : &L->X[k][ib]),
               C = lds_get(ic == 3u ? &L->Z : &L->X[k][ic]);
    fp_t t;
    fp_add(t, A, B);
    fp_sub(x[k], t, C);
  }
  coop_wave_sync();
}

// lazy sum (< 2p), a product input
__device__ __forceinline__ fp_t mkv_lz(const fp_t& a, const fp_t& b) {
  fp_t r;
  fp_add_lazy(r, a, b);
  return r;
}

struct mkv_pair {
  fp_t x, y, z;   // T (homogeneous projective), views
  fp_t xp, yp;    // P (affine G1, full Fp)
};

struct mkv_line {
  fp_t a0, a1, b1;  // l = a0 + a1 w^2 + b1 w^3, views
};

// the tangent step of both pairs (pairing.h miller_dbl_core<true>): rounds
// of 10 and 12 products (the first with f^2 when SQR: see mkv_step)
template <int S>
__device__ __forceinline__ void mkv_dbl_tail(const mkv_grp<S>& g, mkv_pair (&T)[2], mkv_line (&l)[2]) {
  // after round A2: XY, Y^2, Z^2, (Y + Z)^2, X^2 of pair p at 5 p + 0..4
  fp_t A[2], B[2], C[2], W[2], X2[2], E[2], F[2], H[2], G[2], a0[2], x3[2], bf[2];
#pragma unroll
  for (int p = 0; p < 2; p++) {
    A[p] = mkv_get(g, 5 * p);
    B[p] = mkv_get(g, 5 * p + 1);
    C[p] = mkv_get(g, 5 * p + 2);
    W[p] = mkv_get(g, 5 * p + 3);
    X2[p] = mkv_get(g, 5 * p + 4);
  }
  fp_t xc[2] = {C[0], C[1]};
  mkv_xi<S, 2>(g, xc);  // xi Z^2
#pragma unroll
  for (int p = 0; p < 2; p++) {
    fp_half(A[p], A[p]);  // XY / 2
    fp_t t;
    fp_add2(t, xc[p], xc[p], H[p], B[p], C[p]);
    fp_add(t, t, t);       // 4 xi C
    fp_add(E[p], t, t);
    fp_add(E[p], E[p], t);  // 3 b' C = 12 xi C
    fp_add(F[p], E[p], E[p]);
    fp_add(F[p], F[p], E[p]);  // 9 b' C
    fp_sub(H[p], W[p], H[p]);  // 2 YZ
    fp_sub2(a0[p], E[p], B[p], bf[p], B[p], F[p]);
    fp_add(G[p], B[p], F[p]);
    fp_half(G[p], G[p]);  // (Y^2 + 9 b' Z^2) / 2
    fp_add(x3[p], X2[p], X2[p]);
    fp_add(x3[p], x3[p], X2[p]);  // 3 X^2
  }
  // round B: per pair X' = A (B - F), G^2, E^2, Z' = B H, 3X^2 xP, H yP (the last two view-local)
  mkv_round<S, 12, (1u << 4) | (1u << 5) | (1u << 10) | (1u << 11), 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    const int p = j / 6, r = j % 6;
    switch (r) {
      case 0: a = A[p]; b = bf[p]; break;
      case 1: a = G[p]; b = G[p]; break;
      case 2: a = E[p]; b = E[p]; break;
      case 3: a = B[p]; b = H[p]; break;
      case 4: a = x3[p]; b = T[p].xp; break;
      default: a = H[p]; b = T[p].yp; break;
    }
  });
#pragma unroll
  for (int p = 0; p < 2; p++) {
    T[p].x = mkv_get(g, 6 * p);
    const fp_t g2 = mkv_get(g, 6 * p + 1), e2 = mkv_get(g, 6 * p + 2);
    fp_t t;
    fp_add(t, e2, e2);
    fp_add(t, t, e2);
    fp_sub(T[p].y, g2, t);  // G^2 - 3 E^2
    T[p].z = mkv_get(g, 6 * p + 3);
    l[p].a0 = a0[p];
    l[p].a1 = mkv_get(g, 6 * p + 4);
    fp_neg(l[p].b1, mkv_get(g, 6 * p + 5));
  }
}

// the chord step of both pairs with Q_k (pairing.h miller_add_core<true>): 4 rounds
template <int S>
__device__ __forceinline__ void mkv_add(const mkv_grp<S>& g, mkv_pair (&T)[2], const fp_t (&qx)[2],
                                        const fp_t (&qy)[2], mkv_line (&l)[2]) {
  mkv_round<S, 4, 0u, 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    const int p = j >> 1;
    a = (j & 1) ? qx[p] : qy[p];
    b = T[p].z;
  });
  fp_t th[2], la[2];
#pragma unroll
  for (int p = 0; p < 2; p++) fp_sub2(th[p], T[p].y, mkv_get(g, 2 * p), la[p], T[p].x, mkv_get(g, 2 * p + 1));
  // th xQ, la yQ, th^2, la^2, th xP (view-local), la yP (view-local)
  mkv_round<S, 12, (1u << 4) | (1u << 5) | (1u << 10) | (1u << 11), 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    const int p = j / 6, r = j % 6;
    switch (r) {
      case 0: a = th[p]; b = qx[p]; break;
      case 1: a = la[p]; b = qy[p]; break;
      case 2: a = th[p]; b = th[p]; break;
      case 3: a = la[p]; b = la[p]; break;
      case 4: a = th[p]; b = T[p].xp; break;
      default: a = la[p]; b = T[p].yp; break;
    }
  });
  fp_t Cc[2], Dd[2];
#pragma unroll
  for (int p = 0; p < 2; p++) {
    fp_sub(l[p].a0, mkv_get(g, 6 * p), mkv_get(g, 6 * p + 1));
    Cc[p] = mkv_get(g, 6 * p + 2);
    Dd[p] = mkv_get(g, 6 * p + 3);
    fp_neg(l[p].a1, mkv_get(g, 6 * p + 4));
    l[p].b1 = mkv_get(g, 6 * p + 5);
  }
  // E = D la, F = Z C, G = X D
  mkv_round<S, 6, 0u, 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    const int p = j / 3, r = j % 3;
    if (r == 0) { a = Dd[p]; b = la[p]; }
    else if (r == 1) { a = T[p].z; b = Cc[p]; }
    else { a = T[p].x; b = Dd[p]; }
  });
  fp_t E[2], Hh[2], gh[2];
#pragma unroll
  for (int p = 0; p < 2; p++) {
    E[p] = mkv_get(g, 3 * p);
    const fp_t F = mkv_get(g, 3 * p + 1), G = mkv_get(g, 3 * p + 2);
    fp_add(Hh[p], E[p], F);
    fp_sub(Hh[p], Hh[p], G);
    fp_sub(Hh[p], Hh[p], G);
    fp_sub(gh[p], G, Hh[p]);
  }
  // X' = la H, th (G - H), Y E, Z' = Z E
  mkv_round<S, 8, 0u, 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    const int p = j / 4, r = j % 4;
    switch (r) {
      case 0: a = la[p]; b = Hh[p]; break;
      case 1: a = th[p]; b = gh[p]; break;
      case 2: a = T[p].y; b = E[p]; break;
      default: a = T[p].z; b = E[p]; break;
    }
  });
#pragma unroll
  for (int p = 0; p < 2; p++) {
    T[p].x = mkv_get(g, 4 * p);
    fp_sub(T[p].y, mkv_get(g, 4 * p + 1), mkv_get(g, 4 * p + 2));
    T[p].z = mkv_get(g, 4 * p + 3);
  }
}

// l1 l2 = x + y w, x = (k0 + xi k2, k3 - k0 - k1, k1), y = (0, k4 - k0 - k2, k5 - k1 - k2)
// (pairing.h / fp12.h fp12_mul_line2, its first six products)
template <int S>
__device__ __forceinline__ void mkv_lines(const mkv_grp<S>& g, const mkv_line (&l)[2], fp_t (&x)[3], fp_t& y1, fp_t& y2) {
  const mkv_line& u = l[0];
  const mkv_line& v = l[1];
  mkv_round<S, 6, 0u, 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    switch (j) {
      case 0: a = u.a0; b = v.a0; break;
      case 1: a = u.a1; b = v.a1; break;
      case 2: a = u.b1; b = v.b1; break;
      case 3: a = mkv_lz(u.a0, u.a1); b = mkv_lz(v.a0, v.a1); break;
      case 4: a = mkv_lz(u.a0, u.b1); b = mkv_lz(v.a0, v.b1); break;
      default: a = mkv_lz(u.a1, u.b1); b = mkv_lz(v.a1, v.b1); break;
    }
  });
  const fp_t k0 = mkv_get(g, 0), k1 = mkv_get(g, 1), k2 = mkv_get(g, 2), k3 = mkv_get(g, 3), k4 = mkv_get(g, 4),
             k5 = mkv_get(g, 5);
  fp_t xk[1] = {k2};
  mkv_xi<S, 1>(g, xk);
  fp_add(x[0], k0, xk[0]);
  fp_t t;
  fp_sub2(t, k3, k0, y1, k4, k0);
  fp_sub2(x[1], t, k1, y1, y1, k2);
  fp_sub(y2, k5, k1);
  fp_sub(y2, y2, k2);
  x[2] = k1;
}

// f <- f (x + y w), y = (0, y1, y2) (fp12_mul_line2's 6 + 5 + 6 products)
template <int S>
__device__ __forceinline__ void mkv_mul_xy(const mkv_grp<S>& g, fp_t (&fa)[3], fp_t (&fb)[3], const fp_t (&x)[3],
                                           const fp_t& y1, const fp_t& y2) {
  fp_t sa[3], xs[3];
#pragma unroll
  for (int k = 0; k < 3; k++) fp_add(sa[k], fa[k], fb[k]);  // f0 + f1
  xs[0] = x[0];
  fp_add2(xs[1], x[1], y1, xs[2], x[2], y2);  // x + (0, y1, y2)
  // m: f0 x (Karatsuba, m3 xi), n: f1 (y1 v + y2 v^2) (n1..n5 at 6..10, n2 and n3 xi), o: (f0 + f1) xs (o3 xi)
  constexpr uint32_t XI = (1u << 3) | (1u << 7) | (1u << 8) | (1u << 14);
  mkv_round<S, 17, 0u, XI>(g, [&](int j, fp_t& a, fp_t& b) {
    const fp_t* A = j < 6 ? fa : (j < 11 ? fb : sa);
    const fp_t* Bv = j < 6 ? x : xs;
    if (j >= 6 && j < 11) {
      switch (j) {
        case 6: a = fb[1]; b = y1; break;                              // n1 = b1 y1
        case 7: a = fb[2]; b = y2; break;                              // n2 = b2 y2 (xi)
        case 8: a = mkv_lz(fb[1], fb[2]); b = mkv_lz(y1, y2); break;  // n3 (xi)
        case 9: a = fb[0]; b = y1; break;                              // n4 = b0 y1
        default: a = fb[0]; b = y2; break;                             // n5 = b0 y2
      }
      return;
    }
    const int r = j < 6 ? j : j - 11;
    switch (r) {
      case 0: a = A[0]; b = Bv[0]; break;
      case 1: a = A[1]; b = Bv[1]; break;
      case 2: a = A[2]; b = Bv[2]; break;
      case 3: a = mkv_lz(A[1], A[2]); b = mkv_lz(Bv[1], Bv[2]); break;
      case 4: a = mkv_lz(A[0], A[1]); b = mkv_lz(Bv[0], Bv[1]); break;
      default: a = mkv_lz(A[0], A[2]); b = mkv_lz(Bv[0], Bv[2]); break;
    }
  });
  const fp_t m0 = mkv_get(g, 0), m1 = mkv_get(g, 1), m2 = mkv_get(g, 2), xm3 = mkv_get(g, 3), m4 = mkv_get(g, 4),
             m5 = mkv_get(g, 5);
  const fp_t n1 = mkv_get(g, 6), xn2 = mkv_get(g, 7), xn3 = mkv_get(g, 8), n4 = mkv_get(g, 9), n5 = mkv_get(g, 10);
  const fp_t o0 = mkv_get(g, 11), o1 = mkv_get(g, 12), o2 = mkv_get(g, 13), xo3 = mkv_get(g, 14), o4 = mkv_get(g, 15),
             o5 = mkv_get(g, 16);
  fp_t t1c2;
  fp_add(t1c2, n5, n1);  // t1.c2 = b0 y2 + b1 y1
  fp_t xv[6];
  fp_add(xv[0], m1, m2);
  xv[1] = m2;
  xv[2] = n1;
  fp_add(xv[3], o1, o2);
  xv[4] = o2;
  xv[5] = t1c2;
  mkv_xi<S, 6>(g, xv);  // xi (m1 + m2), xi m2, xi n1, xi (o1 + o2), xi o2, xi t1.c2
  // t0 = f0 x: (m0 + xi m3 - xi (m1 + m2), m4 - m0 - m1 + xi m2, m5 - m0 - m2 + m1)
  fp_t t0[3], t1[3], sv[3], u;
  fp_add(u, m0, xm3);
  fp_sub(t0[0], u, xv[0]);
  fp_sub2(u, m4, m0, t0[2], m5, m0);
  fp_sub2(u, u, m1, t0[2], t0[2], m2);
  fp_add2(t0[1], u, xv[1], t0[2], t0[2], m1);
  // t1 = f1 y: (xi n3 - xi n1 - xi n2, n4 + xi n2, n5 + n1)
  fp_sub(u, xn3, xv[2]);
  fp_sub(t1[0], u, xn2);
  fp_add(t1[1], n4, xn2);
  t1[2] = t1c2;
  // sv = (f0 + f1) xs: (o0 + xi o3 - xi (o1 + o2), o4 - o0 - o1 + xi o2, o5 - o0 - o2 + o1)
  fp_add(u, o0, xo3);
  fp_sub(sv[0], u, xv[3]);
  fp_sub2(u, o4, o0, sv[2], o5, o0);
  fp_sub2(u, u, o1, sv[2], sv[2], o2);
  fp_add2(sv[1], u, xv[4], sv[2], sv[2], o1);
  // f1' = sv - t0 - t1, f0' = t0 + v t1 = (t0_0 + xi t1_2, t0_1 + t1_0, t0_2 + t1_1)
#pragma unroll
  for (int k = 0; k < 3; k++) {
    fp_sub(u, sv[k], t0[k]);
    fp_sub(fb[k], u, t1[k]);
  }
  fp_add(fa[0], t0[0], xv[5]);
  fp_add2(fa[1], t0[1], t1[0], fa[2], t0[2], t1[1]);
}

// f <- f^2 (fp12_sqr, complex squaring) in round A1, then the tangent
// products of both pairs in round A2
template <int S>
__device__ __forceinline__ void mkv_sqr(const mkv_grp<S>& g, fp_t (&fa)[3], fp_t (&fb)[3]) {
  fp_t xb[1] = {fb[2]};
  mkv_xi<S, 1>(g, xb);  // xi f1.c2 for h = f0 + v f1
  fp_t gg[3], hh[3];
  fp_add2(gg[0], fa[0], fb[0], gg[1], fa[1], fb[1]);
  fp_add2(gg[2], fa[2], fb[2], hh[0], fa[0], xb[0]);
  fp_add2(hh[1], fa[1], fb[0], hh[2], fa[2], fb[1]);
  // T: f0 f1 (j 0..5, T3 xi), U: g h (j 6..11, U9 xi)
  mkv_round<S, 12, 0u, (1u << 3) | (1u << 9)>(g, [&](int j, fp_t& a, fp_t& b) {
    const fp_t* A = j < 6 ? fa : gg;
    const fp_t* B = j < 6 ? fb : hh;
    switch (j % 6) {
      case 0: a = A[0]; b = B[0]; break;
      case 1: a = A[1]; b = B[1]; break;
      case 2: a = A[2]; b = B[2]; break;
      case 3: a = mkv_lz(A[1], A[2]); b = mkv_lz(B[1], B[2]); break;
      case 4: a = mkv_lz(A[0], A[1]); b = mkv_lz(B[0], B[1]); break;
      default: a = mkv_lz(A[0], A[2]); b = mkv_lz(B[0], B[2]); break;
    }
  });
  const fp_t T0 = mkv_get(g, 0), T1 = mkv_get(g, 1), T2 = mkv_get(g, 2), xT3 = mkv_get(g, 3), T4 = mkv_get(g, 4),
             T5 = mkv_get(g, 5);
  const fp_t U0 = mkv_get(g, 6), U1 = mkv_get(g, 7), U2 = mkv_get(g, 8), xU9 = mkv_get(g, 9), U4 = mkv_get(g, 10),
             U5 = mkv_get(g, 11);
  fp_t t[3], uu[3], w;
  // t2 = T5 - T0 - T2 + T1, u2 likewise
  fp_sub2(t[2], T5, T0, uu[2], U5, U0);
  fp_sub2(t[2], t[2], T2, uu[2], uu[2], U2);
  fp_add2(t[2], t[2], T1, uu[2], uu[2], U1);
  fp_t xv[5];
  fp_add2(xv[0], T1, T2, xv[2], U1, U2);
  xv[1] = T2;
  xv[3] = U2;
  xv[4] = t[2];
  mkv_xi<S, 5>(g, xv);  // xi (T1 + T2), xi T2, xi (U1 + U2), xi U2, xi t2
  fp_add2(t[0], T0, xT3, uu[0], U0, xU9);
  fp_sub2(t[0], t[0], xv[0], uu[0], uu[0], xv[2]);  // T0 + xi (T3 - T1 - T2)
  fp_sub2(t[1], T4, T0, uu[1], U4, U0);
  fp_sub2(t[1], t[1], T1, uu[1], uu[1], U1);
  fp_add2(t[1], t[1], xv[1], uu[1], uu[1], xv[3]);  // T4 - T0 - T1 + xi T2
  // f^2 = (u - t - v t, 2 t), v t = (xi t2, t0, t1)
  fp_sub2(w, uu[0], t[0], fa[1], uu[1], t[1]);
  fp_sub2(fa[0], w, xv[4], fa[1], fa[1], t[0]);
  fp_sub(w, uu[2], t[2]);
  fp_sub(fa[2], w, t[1]);
  fp_add2(fb[0], t[0], t[0], fb[1], t[1], t[1]);
  fp_add(fb[2], t[2], t[2]);
}

// the tangent products of both pairs (round A2)
template <int S>
__device__ __forceinline__ void mkv_dbl_products(const mkv_grp<S>& g, const mkv_pair (&T)[2]) {
  mkv_round<S, 10, 0u, 0u>(g, [&](int j, fp_t& a, fp_t& b) {
    const int p = j / 5, r = j % 5;
    switch (r) {
      case 0: a = T[p].x; b = T[p].y; break;
      case 1: a = T[p].y; b = T[p].y; break;
      case 2: a = T[p].z; b = T[p].z; break;
      case 3: a = mkv_lz(T[p].y, T[p].z); b = a; break;
      default: a = T[p].x; b = T[p].x; break;
    }
  });
}

// the view of 1 and of 0
__device__ __forceinline__ fp_t mkv_one(uint32_t q) {
  fp_t z;
  fp_set_zero(z);
  return q == 1 ? z : FP_ONE;
}

// f = f_{x,Q1}(P1) f_{x,Q2}(P2) for the negative x (conjugated), miller_loop2's
// value.  `two` false: the second pair's lines are replaced by 1 (an odd job's
// last set).  Q views qx, qy per pair; fa / fb: this lane's views of f.
template <int S>
__device__ void mkv_miller2(const mkv_grp<S>& g, mkv_pair (&T)[2], const fp_t (&qx)[2], const fp_t (&qy)[2], bool two,
                            fp_t (&fa)[3], fp_t (&fb)[3]) {
  mkv_line l[2];
  fp_t x[3], y1, y2;
  const fp_t one = mkv_one(g.q);
  fp_t zero;
  fp_set_zero(zero);
  for (int bit = 62; bit >= 0; bit--) {
    if (bit != 62) mkv_sqr<S>(g, fa, fb);
    mkv_dbl_products<S>(g, T);
    mkv_dbl_tail<S>(g, T, l);
    if (!two) { l[1].a0 = one; l[1].a1 = zero; l[1].b1 = zero; }
    mkv_lines<S>(g, l, x, y1, y2);
    if (bit == 62) {  // f = l1 l2
      fa[0] = x[0]; fa[1] = x[1]; fa[2] = x[2];
      fb[0] = zero; fb[1] = y1; fb[2] = y2;
    } else {
      mkv_mul_xy<S>(g, fa, fb, x, y1, y2);
    }
    if ((BLS_X_ABS >> bit) & 1ull) {
      mkv_add<S>(g, T, qx, qy, l);
      if (!two) { l[1].a0 = one; l[1].a1 = zero; l[1].b1 = zero; }
      mkv_lines<S>(g, l, x, y1, y2);
      mkv_mul_xy<S>(g, fa, fb, x, y1, y2);
    }
  }
#pragma unroll
  for (int k = 0; k < 3; k++) fp_neg(fb[k], fb[k]);  // x < 0: conjugate
}

}  // namespace bgv
