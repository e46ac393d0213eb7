// Cooperative G2 arithmetic in Karatsuba VIEWS (latency mode).
//
// A point is worked on by a group of 3 S lanes: S product slots times three
// views.  Lane (s, q) holds, for every Fp2 value x = x0 + x1 i of the point
// formulas, ONE Fp residue, its view q:
//   v0(x) = x0,  v1(x) = x1,  v2(x) = x0 + x1      (canonical, mod p).
// The views are linear, so every addition, subtraction, doubling and negation
// of the formulas is ONE Fp operation per lane (an Fp2 operation on every lane
// of coop_g2.h's layouts is two).  An Fp2 product z = x y is one Fp product
// per view, P_q = v_q(x) v_q(y) (the three Karatsuba sub-products), and after
// one LDS exchange a lane forms its view of z from them:
//   v0(z) = P0 - P1,   v1(z) = P2 - P0 - P1,   v2(z) = P2 - 2 P1,
// with no operand formation before the product (no lazy sums, no component
// selects) and two subtractions after it.  A round computes up to three Fp2
// products: with S = 1 the three views of a group run all of them in turn and
// exchange once; with S = 3 slot s runs product s, combines it, and a second
// exchange hands every lane the views of all of them.  Products by an Fp
// constant stay view-local (psi^2), a product by a conjugate combines the
// sub-products differently (psi).
//
// Every view is a canonical residue, so the Jacobian coordinates are the ones
// curve.h / coop_g2.h compute (same formulas, same order): dbl-2009-l,
// add-2007-bl with the exceptional cases, the 4-bit window, the x-chain and
// Budroni-Pintore h_eff of g2_clear_cofactor, Scott's subgroup test.
// Equality with zero is a wave ballot over views 0 and 1 of slot 0.
#pragma once
#include "miller_coop.h"
#include "lds.h"

namespace bgv {

template <int S>
struct kv_scratch {
  alignas(16) fp_t P[3][4];  // sub-product q of the round's product k; P[k][3] = 0
  alignas(16) fp_t O[3][3];  // S = 3: view q of product k
  alignas(16) fp_t X[4];     // views for the conjugation and the gather; X[3] = 0
};

template <int S>
__device__ __forceinline__ void kv_init(kv_scratch<S>* sc, uint32_t s, uint32_t q) {
  BGV_LDS kv_scratch<S>* L = (BGV_LDS kv_scratch<S>*)sc;
  if (s == 0 && q == 0) {
    fp_t z;
    fp_set_zero(z);
    lds_put(&L->P[0][3], z);
    lds_put(&L->P[1][3], z);
    lds_put(&L->P[2][3], z);
    lds_put(&L->X[3], z);
  }
  coop_wave_sync();
}

// the view of a full Fp2 value on view q
__device__ __forceinline__ fp_t kv_view(const fp2_t& x, uint32_t q) {
  fp_t s;
  fp_add(s, x.c0, x.c1);
  return q == 0 ? x.c0 : (q == 1 ? x.c1 : s);
}

// the combination slots of view q: plain  o = (P[x] - P[y]) - P[z]:  q0 (0, 1, Z)  q1 (2, 0, 1)  q2 (2, 1, 1)
//                                   conj   o = (P[x] + P[y]) - P[z]:  q0 (0, Z, 1)  q1 (0, 1, 2)  q2 (0, 0, 2)
template <bool CONJ>
__device__ __forceinline__ void kv_slots(uint32_t q, uint32_t& ix, uint32_t& iy, uint32_t& iz) {
  if constexpr (!CONJ) {
    ix = q == 0 ? 0u : 2u;
    iy = q == 1 ? 0u : 1u;
    iz = q == 0 ? 3u : 1u;
  } else {
    ix = 0u;
    iy = q == 0 ? 3u : (q == 1 ? 1u : 0u);
    iz = q == 0 ? 1u : 2u;
  }
}

// o_k = a_k * b_k for k < n (n <= 3, a compile-time count after inlining);
// CONJ: o_k = conj(a_k * b_k), whose views are P0 - P1, P0 + P1 - P2, 2 P0 - P2
template <int S, bool CONJ = false>
__device__ __forceinline__ void kv_round(kv_scratch<S>* sc, uint32_t s, uint32_t q, int n, const fp_t& a0,
                                         const fp_t& b0, const fp_t& a1, const fp_t& b1, const fp_t& a2,
                                         const fp_t& b2, fp_t& o0, fp_t& o1, fp_t& o2) {
  BGV_LDS kv_scratch<S>* L = (BGV_LDS kv_scratch<S>*)sc;
  uint32_t ix, iy, iz;
  kv_slots<CONJ>(q, ix, iy, iz);
  if constexpr (S == 1) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k >= n) break;
      fp_t r;
      fp_mul(r, k == 0 ? a0 : (k == 1 ? a1 : a2), k == 0 ? b0 : (k == 1 ? b1 : b2));
      lds_put(&L->P[k][q], r);
    }
    coop_wave_sync();
    // both steps of the n combinations as one interleaved multi-op each (fp_asm.h)
    const fp_t x0 = lds_get(&L->P[0][ix]), y0 = lds_get(&L->P[0][iy]), z0 = lds_get(&L->P[0][iz]);
    if (n == 1) {
      fp_t t;
      if constexpr (!CONJ) fp_sub(t, x0, y0);
      else fp_add(t, x0, y0);
      fp_sub(o0, t, z0);
    } else {
      const fp_t x1 = lds_get(&L->P[1][ix]), y1 = lds_get(&L->P[1][iy]), z1 = lds_get(&L->P[1][iz]);
      if (n == 2) {
        fp_t t0, t1;
        if constexpr (!CONJ) fp_sub2(t0, x0, y0, t1, x1, y1);
        else fp_add2(t0, x0, y0, t1, x1, y1);
        fp_sub2(o0, t0, z0, o1, t1, z1);
      } else {
        const fp_t x2 = lds_get(&L->P[2][ix]), y2 = lds_get(&L->P[2][iy]), z2 = lds_get(&L->P[2][iz]);
        fp_t t0, t1, t2;
        if constexpr (!CONJ) fp_sub3(t0, x0, y0, t1, x1, y1, t2, x2, y2);
        else fp_add3(t0, x0, y0, t1, x1, y1, t2, x2, y2);
        fp_sub3(o0, t0, z0, o1, t1, z1, o2, t2, z2);
      }
    }
    coop_wave_sync();
  } else {
    // slot s: product s (every slot runs one product call: no divergence)
    const fp_t a = s == 0 ? a0 : (s == 1 ? a1 : a2), b = s == 0 ? b0 : (s == 1 ? b1 : b2);
    fp_t r;
    fp_mul(r, a, b);
    if ((int)s < n) lds_put(&L->P[s][q], r);
    coop_wave_sync();
    {
      const uint32_t k = (int)s < n ? s : 0u;
      const fp_t x = lds_get(&L->P[k][ix]), y = lds_get(&L->P[k][iy]), z = lds_get(&L->P[k][iz]);
      fp_t t, o;
      if constexpr (!CONJ) fp_sub(t, x, y);
      else fp_add(t, x, y);
      fp_sub(o, t, z);
      if ((int)s < n) lds_put(&L->O[s][q], o);
    }
    coop_wave_sync();
    o0 = lds_get(&L->O[0][q]);
    if (n > 1) o1 = lds_get(&L->O[1][q]);
    if (n > 2) o2 = lds_get(&L->O[2][q]);
    coop_wave_sync();
  }
}

// conj(x) from the views: v0, -v1, v0 - v1
template <int S>
__device__ __forceinline__ void kv_conj(kv_scratch<S>* sc, uint32_t s, uint32_t q, fp_t& o, const fp_t& x) {
  BGV_LDS kv_scratch<S>* L = (BGV_LDS kv_scratch<S>*)sc;
  if (s == 0) lds_put(&L->X[q], x);
  coop_wave_sync();
  const uint32_t ia = q == 1 ? 3u : 0u, ib = q == 0 ? 3u : 1u;
  const fp_t a = lds_get(&L->X[ia]), b = lds_get(&L->X[ib]);
  fp_sub(o, a, b);
  coop_wave_sync();
}

// x == 0 in Fp2: views 0 and 1 of slot 0 of the group (lanes 3 S grp, +1) are zero
template <int S>
__device__ __forceinline__ bool kv_is_zero(uint32_t grp, const fp_t& v) {
  const uint64_t b = __ballot(fp_is_zero(v));
  return ((b >> (3u * S * grp)) & 3ull) == 3ull;
}

struct kv_pt { fp_t x, y, z; };  // a Jacobian G2 point, this lane's views

__device__ __forceinline__ void kv_load(kv_pt& r, const g2j& p, uint32_t q) {
  r.x = kv_view(p.x, q);
  r.y = kv_view(p.y, q);
  r.z = kv_view(p.z, q);
}

template <int S>
__device__ __forceinline__ bool kv_is_inf(uint32_t grp, const kv_pt& p) { return kv_is_zero<S>(grp, p.z); }

__device__ __forceinline__ void kv_set_inf(kv_pt& r, uint32_t q) {
  // (1, 1, 0) as jac_set_inf: views of 1 are (1, 0, 1)
  const fp_t one = FP_ONE;
  fp_t z;
  fp_set_zero(z);
  r.x = q == 1 ? z : one;
  r.y = q == 1 ? z : one;
  r.z = z;
}

// the group's lane coordinates and scratch
template <int S>
struct kv_grp {
  kv_scratch<S>* sc;
  uint32_t grp, s, q;
};

// dbl-2009-l (coop_g2.h cg_dbl): 3 rounds
template <int S>
__device__ __forceinline__ void kv_dbl(const kv_grp<S>& g, kv_pt& r, const kv_pt& p) {
  fp_t A, B, T, C, Sq, F, E, t, D, x3, G, xb, d;
  kv_round<S>(g.sc, g.s, g.q, 3, p.x, p.x, p.y, p.y, p.y, p.z, A, B, T);
  fp_add2(E, A, A, xb, p.x, B);
  fp_add(E, E, A);  // 3A
  kv_round<S>(g.sc, g.s, g.q, 3, B, B, xb, xb, E, E, C, Sq, F);
  fp_t c2;
  fp_add_sub(c2, C, C, t, Sq, A);
  fp_add_sub(c2, c2, c2, t, t, C);
  fp_add2(c2, c2, c2, D, t, t);  // 8C, D = 2 (Sq - A - C)
  fp_add2(t, D, D, d, T, T);     // 2D, Z3 = 2T
  fp_sub(x3, F, t);
  fp_sub(t, D, x3);
  kv_round<S>(g.sc, g.s, g.q, 1, E, t, E, t, E, t, G, G, G);
  fp_sub(r.y, G, c2);
  r.z = d;
  r.x = x3;
}

// add-2007-bl with the exceptional cases (coop_g2.h cg_add): 6 rounds
template <int S>
__device__ __forceinline__ void kv_add(const kv_grp<S>& g, kv_pt& r, const kv_pt& p, const kv_pt& qq) {
  const bool pi = kv_is_inf<S>(g.grp, p), qi = kv_is_inf<S>(g.grp, qq);
  fp_t z1z1, z2z2, zz, u1, u2, a, b, s1, s2, h, h2, i, j, v, rr, x, z3, x3, y, w, t, zs;
  fp_add(zs, p.z, qq.z);
  kv_round<S>(g.sc, g.s, g.q, 3, p.z, p.z, qq.z, qq.z, zs, zs, z1z1, z2z2, zz);
  kv_round<S>(g.sc, g.s, g.q, 3, p.x, z2z2, qq.x, z1z1, p.y, qq.z, u1, u2, a);
  fp_sub(h, u2, u1);
  fp_dbl(h2, h);
  kv_round<S>(g.sc, g.s, g.q, 3, qq.y, p.z, a, z2z2, h2, h2, b, s1, i);
  kv_round<S>(g.sc, g.s, g.q, 3, b, z1z1, h, i, u1, i, s2, j, v);
  fp_sub2(rr, s2, s1, t, zz, z1z1);
  const bool h0 = kv_is_zero<S>(g.grp, h), r0 = kv_is_zero<S>(g.grp, rr);
  fp_add_sub(rr, rr, rr, t, t, z2z2);
  kv_round<S>(g.sc, g.s, g.q, 2, rr, rr, t, h, t, h, x, z3, z3);
  fp_sub(x3, x, j);
  fp_sub(x3, x3, v);
  fp_sub(x3, x3, v);
  fp_sub(t, v, x3);
  kv_round<S>(g.sc, g.s, g.q, 2, rr, t, s1, j, s1, j, y, w, w);
  fp_dbl(w, w);
  kv_pt sum;
  sum.x = x3;
  fp_sub(sum.y, y, w);
  sum.z = z3;
  // P == Q: the doubling (rare; every lane of the wave takes the branch
  // together so the rounds inside stay wave-wide)
  const bool need_dbl = !pi && !qi && h0 && r0;
  kv_pt d;
  if (__any(need_dbl)) kv_dbl<S>(g, d, p);
  if (pi) r = qq;
  else if (qi) r = p;
  else if (h0) {
    if (r0) r = d;
    else kv_set_inf(r, g.q);
  } else r = sum;
}

__device__ __forceinline__ void kv_neg(kv_pt& r, const kv_pt& p) {
  r.x = p.x;
  fp_neg(r.y, p.y);
  r.z = p.z;
}

// [|x|]P (curve.h jac_mul_abs_x): the bits of |x| are wave-uniform
template <int S>
__device__ void kv_mul_abs_x(const kv_grp<S>& g, kv_pt& r, const kv_pt& p) {
  kv_pt acc = p;
  for (int b = 62; b >= 0; b--) {
    kv_dbl<S>(g, acc, acc);
    if ((BLS_X_ABS >> b) & 1ull) kv_add<S>(g, acc, acc, p);
  }
  r = acc;
}

// psi(P) = (conj(X) cx, conj(Y) cy, conj(Z)) = (conj(X conj(cx)), conj(Y conj(cy)), conj(Z))
template <int S>
__device__ __forceinline__ void kv_psi(const kv_grp<S>& g, kv_pt& r, const kv_pt& p) {
  fp2_t ccx, ccy;
  fp2_conj(ccx, PSI_CX);
  fp2_conj(ccy, PSI_CY);
  const fp_t cx = kv_view(ccx, g.q), cy = kv_view(ccy, g.q);
  fp_t x, y, z;
  kv_round<S, true>(g.sc, g.s, g.q, 2, p.x, cx, p.y, cy, p.y, cy, x, y, y);
  kv_conj<S>(g.sc, g.s, g.q, z, p.z);
  r.x = x;
  r.y = y;
  r.z = z;
}

// psi^2(P) = (X cx2, Y cy2, Z), constants in Fp: view-local products
__device__ __forceinline__ void kv_psi2(kv_pt& r, const kv_pt& p) {
  fp_mul(r.x, p.x, PSI2_CX);
  fp_mul(r.y, p.y, PSI2_CY);
  r.z = p.z;
}

// h_eff [P] (curve.h g2_clear_cofactor, coop_g2.h cg_clear_cofactor)
template <int S>
__device__ void kv_clear_cofactor(const kv_grp<S>& g, kv_pt& r, const kv_pt& p) {
  kv_pt t1, t2, t3, np;
  kv_mul_abs_x<S>(g, t1, p);
  kv_neg(t1, t1);  // [x]P
  kv_mul_abs_x<S>(g, t2, t1);
  kv_neg(t2, t2);  // [x^2]P
  kv_neg(np, p);
  kv_add<S>(g, t3, t1, np);  // [x - 1]P
  kv_psi<S>(g, t3, t3);
  kv_neg(t1, t1);
  kv_add<S>(g, t2, t2, t1);  // [x^2 - x]P
  kv_add<S>(g, t2, t2, np);  // [x^2 - x - 1]P
  kv_add<S>(g, t2, t2, t3);
  kv_dbl<S>(g, t1, p);
  kv_psi2(t1, t1);
  kv_add<S>(g, r, t2, t1);
}

// equality of two Jacobian points (curve.h jac_eq, cross-multiplied)
template <int S>
__device__ __forceinline__ bool kv_eq(const kv_grp<S>& g, const kv_pt& p, const kv_pt& qq) {
  const bool pi = kv_is_inf<S>(g.grp, p), qi = kv_is_inf<S>(g.grp, qq);
  fp_t z1z1, z2z2, a, b, c, d, e;
  kv_round<S>(g.sc, g.s, g.q, 3, p.z, p.z, qq.z, qq.z, p.y, qq.z, z1z1, z2z2, c);
  kv_round<S>(g.sc, g.s, g.q, 3, p.x, z2z2, qq.x, z1z1, qq.y, p.z, a, b, d);
  kv_round<S>(g.sc, g.s, g.q, 2, c, z2z2, d, z1z1, d, z1z1, c, d, d);
  fp_sub2(e, a, b, c, c, d);
  const bool ex = kv_is_zero<S>(g.grp, e), ey = kv_is_zero<S>(g.grp, c);
  if (pi || qi) return pi && qi;
  return ex && ey;
}

// Scott's test psi(P) == [x]P (curve.h g2_in_subgroup)
template <int S>
__device__ bool kv_in_subgroup(const kv_grp<S>& g, const kv_pt& p) {
  kv_pt xp, ps;
  kv_mul_abs_x<S>(g, xp, p);
  kv_neg(xp, xp);
  kv_psi<S>(g, ps, p);
  const bool eq = kv_eq<S>(g, ps, xp);
  return kv_is_inf<S>(g.grp, p) || eq;
}

// [k]P, 4-bit fixed window (curve.h jac_mul_u64_w4); the table (16 points)
// sits in LDS as full Jacobian points: views 0 and 1 of slot 0 write their
// components, every lane forms its view on reading (view 2 = c0 + c1)
template <int S>
__device__ void kv_mul_u64_w4(const kv_grp<S>& g, g2j* tab, bool lead, kv_pt& r, const kv_pt& p, uint64_t k) {
  BGV_LDS g2j* T = (BGV_LDS g2j*)tab;
  const bool wr = lead && g.s == 0 && g.q < 2;
  auto put = [&](int i, const kv_pt& v) {
    if (wr) {
      lds_put(g.q ? &T[i].x.c1 : &T[i].x.c0, v.x);
      lds_put(g.q ? &T[i].y.c1 : &T[i].y.c0, v.y);
      lds_put(g.q ? &T[i].z.c1 : &T[i].z.c0, v.z);
    }
  };
  auto get = [&](uint32_t i) {
    const fp_t x0 = lds_get(&T[i].x.c0), x1 = lds_get(&T[i].x.c1), y0 = lds_get(&T[i].y.c0),
               y1 = lds_get(&T[i].y.c1), z0 = lds_get(&T[i].z.c0), z1 = lds_get(&T[i].z.c1);
    fp_t sx, sy, sz;
    fp_add3(sx, x0, x1, sy, y0, y1, sz, z0, z1);
    kv_pt v;
    v.x = g.q == 0 ? x0 : (g.q == 1 ? x1 : sx);
    v.y = g.q == 0 ? y0 : (g.q == 1 ? y1 : sy);
    v.z = g.q == 0 ? z0 : (g.q == 1 ? z1 : sz);
    return v;
  };
  kv_pt t;
  kv_set_inf(t, g.q);
  put(0, t);
  put(1, p);
  kv_dbl<S>(g, t, p);
  put(2, t);
#pragma unroll 1
  for (int i = 3; i < 16; i++) {
    kv_add<S>(g, t, t, p);
    put(i, t);
  }
  coop_wave_sync();
  kv_pt acc = get((uint32_t)(k >> 60) & 15u);
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    kv_dbl<S>(g, acc, acc);
    kv_dbl<S>(g, acc, acc);
    kv_dbl<S>(g, acc, acc);
    kv_dbl<S>(g, acc, acc);
    const kv_pt e = get((uint32_t)(k >> (4 * w)) & 15u);
    kv_add<S>(g, acc, acc, e);
  }
  r = acc;
}

// the whole point on slot 0, view 0 (views 0 and 1 are the components)
template <int S>
__device__ __forceinline__ void kv_gather(const kv_grp<S>& g, g2j& out, const kv_pt& p) {
  BGV_LDS kv_scratch<S>* L = (BGV_LDS kv_scratch<S>*)g.sc;
  const fp_t* c[3] = {&p.x, &p.y, &p.z};
  fp2_t* o[3] = {&out.x, &out.y, &out.z};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (g.s == 0 && g.q < 2) lds_put(&L->X[g.q], *c[k]);
    coop_wave_sync();
    o[k]->c0 = lds_get(&L->X[0]);
    o[k]->c1 = lds_get(&L->X[1]);
    coop_wave_sync();
  }
}

}  // namespace bgv
