// Fp12 arithmetic spread over a 128-thread workgroup (two waves), one Fp
// product per lane: the latency-bound tail of the verifier (per-job folds of
// the Miller values, the batch product, the final exponentiations) runs at
// the latency of ONE Fp product per Fp12 multiplication.
//
// Same basis as fp12_wave.h: Fp12 = Fp2[w] / (w^6 - xi), w^k coefficient k
// (tower slot: 0 c0.c0, 1 c1.c0, 2 c0.c1, 3 c1.c1, 4 c0.c2, 5 c1.c2).  A
// product a * b is the 6 x 6 schoolbook of Fp2 products a_i b_j, each by
// Karatsuba over three Fp products:
//   round 1  lane l < 108: pair p = l / 3 (i = p / 6, j = p % 6), Fp product
//            q = l % 3 of a_i b_j: a0 b0 | a1 b1 | (a0 + a1)(b0 + b1)
//   round 2  lane l < 36: a_i b_j = (P0 - P1) + (P2 - P0 - P1) i, times xi
//            when i + j >= 6
//   round 3  lane l < 12: one Fp component of c_k = sum_i a_i b_(k-i)
// Every function is called by all 128 threads (it contains __syncthreads()).
#pragma once
#include "fp12_wave.h"
#include "lds.h"

namespace bgv {

constexpr uint32_t COOP_THREADS = 128;

struct cscratch {
  fp_t p[108];
  fp2_t q[36];
  wfp12 t[6];  // temporaries of the final exponentiation
};

// out = a * b (out may alias a or b)
#ifndef BGV_COOP_LDS_AS
#define BGV_COOP_LDS_AS 1
#endif
#ifndef BGV_COOP_TREE
#define BGV_COOP_TREE 1  // c_mul2: the output sums across lanes instead of a third round
#endif
#ifndef BGV_CMUL_ADDR
#define BGV_CMUL_ADDR 1
#endif
#if BGV_COOP_LDS_AS && BGV_COOP_TREE
// out = a * b in TWO rounds: the 108 Fp products, then one Fp component per
// lane (wave c = component c): lane m = 6k + i takes the product pair
// (i, k - i mod 6), and the six terms of c_k sum across lanes 6k .. 6k + 5
// (ds_bpermute, no barrier) as ((t0 + t1) + (t2 + t3)) + (t4 + t5)
// value of v in lane src of this wave (ds_bpermute addresses lanes within the wave)
__device__ __forceinline__ fp_t c_pull1(const fp_t& v, uint32_t src) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < NL; k++) r.l[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v.l[k]);
  return r;
}
__device__ void c_mul(wfp12* out_, const wfp12* a_, const wfp12* b_, cscratch* s_) {
  BGV_LDS wfp12* out = (BGV_LDS wfp12*)out_;
  const BGV_LDS wfp12* a = (const BGV_LDS wfp12*)a_;
  const BGV_LDS wfp12* b = (const BGV_LDS wfp12*)b_;
  BGV_LDS cscratch* s = (BGV_LDS cscratch*)s_;
  const uint32_t l = threadIdx.x;
  if (l < 108) {
    const uint32_t p = l / 3, q = l - 3 * p, i = p / 6, j = p - 6 * i;
    fp_t u, v;
#if BGV_CMUL_ADDR
    // operands by address, not by value selects: component q (q < 2) or c0,
    // plus c1 masked in for the Karatsuba sum (q = 2; a lazy sum of x and 0
    // is x), so every lane runs one load pair and one lazy addition
    const uint32_t m = q == 2 ? ~0u : 0u;
    const fp_t xa = lds_get(q == 1 ? &a->c[i].c1 : &a->c[i].c0), ya = lds_get(&a->c[i].c1);
    const fp_t xb = lds_get(q == 1 ? &b->c[j].c1 : &b->c[j].c0), yb = lds_get(&b->c[j].c1);
    fp_t ma, mb;
#pragma unroll
    for (int k = 0; k < NL; k++) {
      ma.l[k] = ya.l[k] & m;
      mb.l[k] = yb.l[k] & m;
    }
    fp_add_lazy2(u, xa, ma, v, xb, mb);
#else
    if (q == 0) {
      u = lds_get(&a->c[i].c0);
      v = lds_get(&b->c[j].c0);
    } else if (q == 1) {
      u = lds_get(&a->c[i].c1);
      v = lds_get(&b->c[j].c1);
    } else {
      fp_add_lazy2(u, lds_get(&a->c[i].c0), lds_get(&a->c[i].c1), v, lds_get(&b->c[j].c0), lds_get(&b->c[j].c1));
    }
#endif
    fp_t r;
    fp_mul(r, u, v);
    lds_put(&s->p[l], r);
  }
  __syncthreads();
  {
    // round 2, one Fp component per lane: wave comp (0 or 1) handles component
    // comp of every output coefficient; lane m = 6k + i of the wave takes the
    // product pair (i, j = k - i mod 6), whose Fp2 value is (P0 - P1) + (P2 - P0 - P1) u,
    // times xi when i + j >= 6:  re: 2 P0 - P2,  im: P2 - 2 P1.  Its component is
    // one addition and one subtraction, the six terms of c_k then sum across the
    // lanes (ds_bpermute) as ((t0 + t1) + (t2 + t3)) + (t4 + t5)
    const uint32_t comp = l >> 6, m = l & 63u;
    const uint32_t k = m / 6 < 6 ? m / 6 : 0u, i = m % 6, j = (k + 6 - i) % 6, pr = i * 6 + j;
    const bool xi = i + j >= 6;
    // w = a + b;  t = c - d
    //   re, no xi: (P0 + 0) - P1     re, xi: (P0 + P0) - P2
    //   im, no xi: P2 - (P0 + P1)    im, xi: P2 - (P1 + P1)
#if BGV_CMUL_ADDR
    // a, b and the other term Q by address (b masked to 0 for re without xi):
    // re: t = w - Q, im: t = Q - w
    const uint32_t mb = comp || xi ? ~0u : 0u;
    const fp_t a = lds_get(&s->p[3 * pr + (comp && xi ? 1u : 0u)]);
    const fp_t b0 = lds_get(&s->p[3 * pr + (comp ? 1u : 0u)]);
    const fp_t Q = lds_get(&s->p[3 * pr + (comp || xi ? 2u : 1u)]);
    fp_t b;
#pragma unroll
    for (int k = 0; k < NL; k++) b.l[k] = b0.l[k] & mb;
    fp_t w, t;
    fp_add(w, a, b);
    fp_sub(t, comp ? Q : w, comp ? w : Q);
#else
    const fp_t p0 = lds_get(&s->p[3 * pr]), p1 = lds_get(&s->p[3 * pr + 1]), p2 = lds_get(&s->p[3 * pr + 2]);
    fp_t zero;
    fp_set_zero(zero);
    const fp_t& a = comp ? (xi ? p1 : p0) : p0;
    const fp_t& b = comp ? p1 : (xi ? p0 : zero);
    fp_t w, t;
    fp_add(w, a, b);
    fp_sub(t, comp ? p2 : w, comp ? w : (xi ? p2 : p1));
#endif
    const uint32_t src1 = m + 1 < 64 ? l + 1 : l, src2 = m + 2 < 64 ? l + 2 : l, src4 = m + 4 < 64 ? l + 4 : l;
    fp_t x = c_pull1(t, src1 & 63u);  // i even: t_i + t_(i+1)
    fp_add(t, t, x);
    x = c_pull1(t, src2 & 63u);        // i = 0: (t0 + t1) + (t2 + t3)
    const fp_t y = c_pull1(t, src4 & 63u);  // i = 0: t4 + t5
    fp_add(t, t, x);
    fp_add(t, t, y);
    if (m < 36 && i == 0) lds_put(comp ? &out->c[k].c1 : &out->c[k].c0, t);
  }
  __syncthreads();
}
#elif BGV_COOP_LDS_AS
// c_mul is a non-inlined function whose operands all live in LDS: the
// casts below make its accesses ds_read / ds_write (lds.h)
__device__ void c_mul(wfp12* out_, const wfp12* a_, const wfp12* b_, cscratch* s_) {
  BGV_LDS wfp12* out = (BGV_LDS wfp12*)out_;
  const BGV_LDS wfp12* a = (const BGV_LDS wfp12*)a_;
  const BGV_LDS wfp12* b = (const BGV_LDS wfp12*)b_;
  BGV_LDS cscratch* s = (BGV_LDS cscratch*)s_;
  const uint32_t l = threadIdx.x;
  if (l < 108) {
    const uint32_t p = l / 3, q = l - 3 * p, i = p / 6, j = p - 6 * i;
    fp_t u, v;
    if (q == 0) {
      u = lds_get(&a->c[i].c0);
      v = lds_get(&b->c[j].c0);
    } else if (q == 1) {
      u = lds_get(&a->c[i].c1);
      v = lds_get(&b->c[j].c1);
    } else {
      fp_add_lazy(u, lds_get(&a->c[i].c0), lds_get(&a->c[i].c1));  // < 2p, product inputs only
      fp_add_lazy(v, lds_get(&b->c[j].c0), lds_get(&b->c[j].c1));
    }
    fp_t r;
    fp_mul(r, u, v);
    lds_put(&s->p[l], r);
  }
  __syncthreads();
  if (l < 36) {
    const uint32_t i = l / 6, j = l - 6 * i;
    const fp_t p0 = lds_get(&s->p[3 * l]), p1 = lds_get(&s->p[3 * l + 1]), p2 = lds_get(&s->p[3 * l + 2]);
    fp2_t t;
    fp_t w;
    fp_add_sub(w, p0, p1, t.c0, p0, p1);
    fp_sub(t.c1, p2, w);
    if (i + j >= 6) fp2_mul_xi(t, t);
    lds_put(&s->q[l].c0, t.c0);
    lds_put(&s->q[l].c1, t.c1);
  }
  __syncthreads();
  if (l < 12) {
    const uint32_t k = l >> 1, comp = l & 1;
    // c_k = sum_i q[i][k - i]: a tree of dual additions, ((t0 + t1) + (t2 + t3)) + (t4 + t5)
    fp_t t[6];
#pragma unroll
    for (uint32_t i = 0; i < 6; i++) {
      const BGV_LDS fp2_t* e = &s->q[i * 6 + (k + 6 - i) % 6];
      t[i] = lds_get(comp ? &e->c1 : &e->c0);
    }
    fp_t s01, s23, s45, acc;
    fp_add2(s01, t[0], t[1], s23, t[2], t[3]);
    fp_add2(s45, t[4], t[5], acc, s01, s23);
    fp_add(acc, acc, s45);
    lds_put(comp ? &out->c[k].c1 : &out->c[k].c0, acc);
  }
  __syncthreads();
}
#else
__device__ void c_mul(wfp12* out, const wfp12* a, const wfp12* b, cscratch* s) {
  const uint32_t l = threadIdx.x;
  if (l < 108) {
    const uint32_t p = l / 3, q = l - 3 * p, i = p / 6, j = p - 6 * i;
    const fp2_t& x = a->c[i];
    const fp2_t& y = b->c[j];
    fp_t u, v;
    if (q == 0) {
      u = x.c0;
      v = y.c0;
    } else if (q == 1) {
      u = x.c1;
      v = y.c1;
    } else {
      fp_add_lazy(u, x.c0, x.c1);  // < 2p, product inputs only
      fp_add_lazy(v, y.c0, y.c1);
    }
    fp_mul(s->p[l], u, v);
  }
  __syncthreads();
  if (l < 36) {
    const uint32_t i = l / 6, j = l - 6 * i;
    fp2_t t;
    fp_t w;
    fp_sub(t.c0, s->p[3 * l], s->p[3 * l + 1]);
    fp_add(w, s->p[3 * l], s->p[3 * l + 1]);
    fp_sub(t.c1, s->p[3 * l + 2], w);
    if (i + j >= 6) fp2_mul_xi(t, t);
    s->q[l] = t;
  }
  __syncthreads();
  if (l < 12) {
    const uint32_t k = l >> 1, comp = l & 1;
    fp_t acc = comp ? s->q[k].c1 : s->q[k].c0;  // i = 0, j = k
#pragma unroll
    for (uint32_t i = 1; i < 6; i++) {
      const fp2_t& t = s->q[i * 6 + (k + 6 - i) % 6];
      fp_add(acc, acc, comp ? t.c1 : t.c0);
    }
    if (comp) out->c[k].c1 = acc;
    else out->c[k].c0 = acc;
  }
  __syncthreads();
}
#endif

// acc = acc^2 for acc in the cyclotomic subgroup (after the easy part of the
// final exponentiation): Granger-Scott over Fp4 = Fp2[s]/(s^2 - xi), s = w^3,
// with fp12_cyclotomic_sqr's formulas (fp12.h) and pairs (w^p, w^(p+3)),
// p = 0, 1, 2.  Its nine Fp2 squarings are one Fp squaring per lane in
// Karatsuba views (kv_g2.h), so a squaring is one product deep instead of
// c_mul's 108-product round and cross-lane sum.  Wave 0 only:
//   R1 lane 3m + q (m < 9): pair p = m / 3, x = a | b | a + b (m % 3),
//      P[m][q] = v_q(x)^2 with v0 = x0, v1 = x1, v2 = x0 + x1
//   R2 lane 2m + c (m < 9): component c of x_m^2: P0 - P1 | P2 - (P0 + P1)
//   R3 lane 2k + c (k < 6): component c of w^k' = 3 t_k -+ 2 w^k with
//      t = a^2 + xi b^2 of pair k / 2 (k even, minus), (a + b)^2 - a^2 - b^2
//      of pair 0 (k = 3) or 1 (k = 5), xi times it of pair 2 (k = 1) (plus)
// Canonical residues in and out: bit-identical to c_mul(acc, acc, acc) (GPU
// stage tests green with it on).  Off: a lone wave's latency is its
// instruction count, and the squaring's linear combinations (R3: up to seven
// modular multi-ops and the operand selects on one lane) cost about what
// c_mul's 108-lane round and cross-lane sum do: k_batch_final 1.20-1.39 ms
// with it against 1.23-1.27 without (r04, profiles/r04c_ab_fe_cyc.txt).
#ifndef BGV_FE_CYC
#define BGV_FE_CYC 0
#endif
__device__ __forceinline__ void c_wave_fence() { __builtin_amdgcn_wave_barrier(); __asm__ volatile("" ::: "memory"); }
__device__ void c_cyc_sqr(wfp12* acc_, cscratch* s_) {
  BGV_LDS wfp12* acc = (BGV_LDS wfp12*)acc_;
  BGV_LDS cscratch* s = (BGV_LDS cscratch*)s_;
  const uint32_t l = threadIdx.x;
  if (l < 64) {
    if (l < 27) {
      const uint32_t m = l / 3, q = l - 3 * m, p = m / 3, kind = m - 3 * p;
      const fp_t a0 = lds_get(&acc->c[p].c0), a1 = lds_get(&acc->c[p].c1);
      const fp_t b0 = lds_get(&acc->c[p + 3].c0), b1 = lds_get(&acc->c[p + 3].c1);
      fp_t s0, s1;
      fp_add2(s0, a0, b0, s1, a1, b1);
      const fp_t& x0 = kind == 0 ? a0 : (kind == 1 ? b0 : s0);
      const fp_t& x1 = kind == 0 ? a1 : (kind == 1 ? b1 : s1);
      fp_t v2;
      fp_add_lazy(v2, x0, x1);  // < 2p, product input only
      const fp_t& v = q == 0 ? x0 : (q == 1 ? x1 : v2);
      fp_t r;
      fp_sqr(r, v);
      lds_put(&s->p[l], r);
    }
    c_wave_fence();
    if (l < 18) {
      const uint32_t m = l >> 1, c = l & 1u;
      const fp_t p0 = lds_get(&s->p[3 * m]), p1 = lds_get(&s->p[3 * m + 1]), p2 = lds_get(&s->p[3 * m + 2]);
      fp_t w;
      fp_add(w, p0, p1);
      fp_t r;
      fp_sub(r, c ? p2 : p0, c ? w : p1);
      lds_put(c ? &s->q[m].c1 : &s->q[m].c0, r);
    }
    c_wave_fence();
    if (l < 12) {
      const uint32_t k = l >> 1, c = l & 1u;
      const bool odd = k & 1u;
      // squares of the pair: A = a^2, B = b^2, C = (a + b)^2 (both components)
      const uint32_t pr = odd ? (k == 3 ? 0u : (k == 5 ? 1u : 2u)) : k >> 1;
      const fp2_t A = {lds_get(&s->q[3 * pr].c0), lds_get(&s->q[3 * pr].c1)};
      const fp2_t B = {lds_get(&s->q[3 * pr + 1].c0), lds_get(&s->q[3 * pr + 1].c1)};
      const fp2_t C = {lds_get(&s->q[3 * pr + 2].c0), lds_get(&s->q[3 * pr + 2].c1)};
      fp_t t;
      if (!odd) {  // (a^2 + xi b^2)_c = A_c + (B0 -+ B1)
        fp_t bs, bd;
        fp_add_sub(bs, B.c0, B.c1, bd, B.c0, B.c1);
        fp_add(t, c ? A.c1 : A.c0, c ? bs : bd);
      } else {  // r = C - A - B; t = r_c, or (xi r)_c = r0 -+ r1 for k = 1
        fp_t u0, u1, r0, r1;
        fp_add2(u0, A.c0, B.c0, u1, A.c1, B.c1);
        fp_sub2(r0, C.c0, u0, r1, C.c1, u1);
        fp_t xs, xd;
        fp_add_sub(xs, r0, r1, xd, r0, r1);
        t = k == 1 ? (c ? xs : xd) : (c ? r1 : r0);
      }
      // 3 t - 2 z (k even) or 3 t + 2 z (k odd) = 2 (t -+ z) + t
      const fp_t z = lds_get(c ? &acc->c[k].c1 : &acc->c[k].c0);
      fp_t ts, td;
      fp_add_sub(ts, t, z, td, t, z);
      fp_t u = odd ? ts : td, o;
      fp_add(u, u, u);
      fp_add(o, u, t);
      lds_put(c ? &acc->c[k].c1 : &acc->c[k].c0, o);
    }
  }
  __syncthreads();
}

__device__ void c_set_one(wfp12* r) {
  const uint32_t l = threadIdx.x;
  if (l < 6) r->c[l] = l == 0 ? fp2_one() : fp2_zero();
  __syncthreads();
}

// r = f (tower layout, any address space) in the w basis
__device__ void c_load(wfp12* r, const fp12_t& f) {
  const uint32_t l = threadIdx.x;
  if (l < 6) {
    const fp6_t& h = (l & 1) ? f.c1 : f.c0;
    const uint32_t s = l >> 1;
    r->c[l] = s == 0 ? h.c0 : (s == 1 ? h.c1 : h.c2);
  }
  __syncthreads();
}

__device__ void c_store(fp12_t& f, const wfp12* r) {
  const uint32_t l = threadIdx.x;
  if (l < 6) {
    fp6_t& h = (l & 1) ? f.c1 : f.c0;
    const uint32_t s = l >> 1;
    if (s == 0) h.c0 = r->c[l];
    else if (s == 1) h.c1 = r->c[l];
    else h.c2 = r->c[l];
  }
  __syncthreads();
}

__device__ void c_copy(wfp12* out, const wfp12* a) {
  const uint32_t l = threadIdx.x;
  if (l < 6) out->c[l] = a->c[l];
  __syncthreads();
}

__device__ void c_conj(wfp12* out, const wfp12* a) {
  const uint32_t l = threadIdx.x;
  if (l < 6) {
    fp2_t t = a->c[l];
    if (l & 1) fp2_neg(t, t);
    out->c[l] = t;
  }
  __syncthreads();
}

// Frobenius pi^k, k = 1..3: lane 2m + c computes component c of coefficient m
__device__ void c_frob(wfp12* out, const wfp12* a, int k, cscratch* s) {
  const uint32_t l = threadIdx.x;
  if (l < 12) {
    const uint32_t m = l >> 1, comp = l & 1;
    fp2_t t = a->c[m];
    if (k & 1) fp2_conj(t, t);
    fp_t r;
    if (m == 0) {
      r = comp ? t.c1 : t.c0;
    } else {  // (t0 + t1 i)(g0 + g1 i): component comp by two Fp products, the same
              // instruction stream on both components (operands selected, no branch)
      const fp2_t& g = FROB_G[k - 1][m - 1];
      fp_t x, y, sum, diff;
      fp_mul(x, t.c0, comp ? g.c1 : g.c0);
      fp_mul(y, t.c1, comp ? g.c0 : g.c1);
      fp_add_sub(sum, x, y, diff, x, y);
      r = comp ? sum : diff;
    }
    s->p[l] = r;
  }
  __syncthreads();
  if (l < 6) {
    out->c[l].c0 = s->p[2 * l];
    out->c[l].c1 = s->p[2 * l + 1];
  }
  __syncthreads();
}

// out = a^x (x < 0) for a in the cyclotomic subgroup
__device__ void c_pow_x(wfp12* out, const wfp12* a, wfp12* acc, cscratch* s) {
  c_copy(acc, a);
  for (int b = 62; b >= 0; b--) {
#if BGV_FE_CYC
    c_cyc_sqr(acc, s);
#else
    c_mul(acc, acc, acc, s);
#endif
    if ((BLS_X_ABS >> b) & 1ull) c_mul(acc, acc, a, s);
  }
  c_conj(out, acc);
}

// Final exponentiation with the addition chain of fp12_final_exp: out (in
// LDS, tower form) = f^(3 (p^12 - 1) / r), the cube of the textbook value
// (the hard-part chain computes m^(3 (p^4 - p^2 + 1) / r); 3 is prime to r,
// so the value is 1 exactly when the textbook one is).
// Karatsuba Fp6 product terms of x * y (tower Fp6 = Fp2[v]/(v^3 - xi)):
// term k of {x0 y0, x1 y1, x2 y2, (x1+x2)(y1+y2), (x0+x1)(y0+y1), (x0+x2)(y0+y2)}
__device__ __forceinline__ void c6_term(fp2_t& r, const fp6_t& x, const fp6_t& y, uint32_t k) {
  fp2_t a, b;
  if (k < 3) {
    a = k == 0 ? x.c0 : (k == 1 ? x.c1 : x.c2);
    b = k == 0 ? y.c0 : (k == 1 ? y.c1 : y.c2);
  } else {
    const fp2_t& xa = k == 5 ? x.c0 : (k == 3 ? x.c1 : x.c0);
    const fp2_t& xb = k == 3 ? x.c2 : (k == 4 ? x.c1 : x.c2);
    const fp2_t& ya = k == 5 ? y.c0 : (k == 3 ? y.c1 : y.c0);
    const fp2_t& yb = k == 3 ? y.c2 : (k == 4 ? y.c1 : y.c2);
    fp2_add(a, xa, xb);
    fp2_add(b, ya, yb);
  }
  fp2_mul(r, a, b);
}
// the Karatsuba recombination of fp6_mul from its six terms
__device__ __forceinline__ void c6_combine(fp6_t& r, const fp2_t* t) {
  fp2_t u, x;
  fp2_sub(u, t[3], t[1]);
  fp2_sub(u, u, t[2]);
  fp2_mul_xi(u, u);
  fp2_add(r.c0, u, t[0]);
  fp2_sub(u, t[4], t[0]);
  fp2_sub(u, u, t[1]);
  fp2_mul_xi(x, t[2]);
  fp2_add(r.c1, u, x);
  fp2_sub(u, t[5], t[0]);
  fp2_sub(u, u, t[2]);
  fp2_add(r.c2, u, t[1]);
}

// Fp12 inversion over the workgroup (fp12_inv's formulas and values): the
// Fp2 products of each level on separate lanes, the recombinations on few,
// the one Fp inversion (divsteps) on lane 0.  ~8 product levels instead of
// ~100 sequential products on one lane (263 us, tools/ubench_coop.hip).
//   1 / (a0 + a1 w) = (a0 - a1 w) / (a0^2 - v a1^2)
struct cinv_scratch {
  fp6_t a0, a1, t, c, ti, r0, r1;
  fp2_t n, ni;
  fp_t nn;
};
__device__ void c_inv12(fp12_t* out, const fp12_t& f, cinv_scratch* v, cscratch* s) {
  const uint32_t l = threadIdx.x;
  fp2_t* q = s->q;  // 36 Fp2 slots
  if (l == 0) { v->a0 = f.c0; v->a1 = f.c1; }
  __syncthreads();
  // a0^2 and a1^2: 12 Karatsuba terms
  if (l < 12) c6_term(q[l], l < 6 ? v->a0 : v->a1, l < 6 ? v->a0 : v->a1, l % 6);
  __syncthreads();
  if (l == 0) {
    fp6_t t0, t1;
    c6_combine(t0, q);
    c6_combine(t1, q + 6);
    fp6_mul_v(t1, t1);
    fp6_sub(v->t, t0, t1);
  }
  __syncthreads();
  // fp6_inv: c0 = t0^2 - xi t1 t2, c1 = xi t2^2 - t0 t1, c2 = t1^2 - t0 t2
  if (l < 6) {
    const fp2_t* x[6] = {&v->t.c0, &v->t.c1, &v->t.c2, &v->t.c0, &v->t.c1, &v->t.c0};
    const fp2_t* y[6] = {&v->t.c0, &v->t.c2, &v->t.c2, &v->t.c1, &v->t.c1, &v->t.c2};
    fp2_mul(q[l], *x[l], *y[l]);
  }
  __syncthreads();
  if (l < 3) {
    fp2_t r, u;
    if (l == 0) { fp2_mul_xi(u, q[1]); fp2_sub(r, q[0], u); v->c.c0 = r; }
    else if (l == 1) { fp2_mul_xi(u, q[2]); fp2_sub(r, u, q[3]); v->c.c1 = r; }
    else { fp2_sub(r, q[4], q[5]); v->c.c2 = r; }
  }
  __syncthreads();
  // n = t0 c0 + xi (t2 c1 + t1 c2)
  if (l < 3) {
    const fp2_t* x[3] = {&v->t.c2, &v->t.c1, &v->t.c0};
    const fp2_t* y[3] = {&v->c.c1, &v->c.c2, &v->c.c0};
    fp2_mul(q[l], *x[l], *y[l]);
  }
  __syncthreads();
  if (l == 0) {
    fp2_t n, u;
    fp2_add(u, q[0], q[1]);
    fp2_mul_xi(u, u);
    fp2_add(n, u, q[2]);
    v->n = n;
    // fp2_inv: n^-1 = conj(n) / (n0^2 + n1^2)
    fp_t nn;
    fp2_norm(nn, n);
    fp_inv(nn, nn);
    v->nn = nn;
  }
  __syncthreads();
  if (l < 2) {
    fp_t r;
    fp_mul(r, l == 0 ? v->n.c0 : v->n.c1, v->nn);
    if (l == 0) v->ni.c0 = r;
    else fp_neg(v->ni.c1, r);
  }
  __syncthreads();
  // t^-1 = c * n^-1
  if (l < 3) fp2_mul(l == 0 ? v->ti.c0 : (l == 1 ? v->ti.c1 : v->ti.c2), l == 0 ? v->c.c0 : (l == 1 ? v->c.c1 : v->c.c2), v->ni);
  __syncthreads();
  // a0 t^-1 and a1 t^-1: 12 Karatsuba terms
  if (l < 12) c6_term(q[l], l < 6 ? v->a0 : v->a1, v->ti, l % 6);
  __syncthreads();
  if (l < 2) {
    fp6_t r;
    c6_combine(r, q + 6 * l);
    if (l == 0) out->c0 = r;
    else fp6_neg(out->c1, r);
  }
  __syncthreads();
}

__device__ void c_final_exp(fp12_t* out, const fp12_t& f_in, cscratch* s) {
  const uint32_t l = threadIdx.x;
  wfp12 *t0 = &s->t[0], *t1 = &s->t[1], *y0 = &s->t[2], *y1 = &s->t[3], *y2 = &s->t[4], *acc = &s->t[5];
  __shared__ wfp12 fin, y3;
  __shared__ cinv_scratch iv;
  __shared__ fp12_t inv;
  c_inv12(&inv, f_in, &iv, s);
  if (l == 0) {
    w_from_tower(*t0, inv);
    w_from_tower(fin, f_in);
  }
  __syncthreads();
  c_conj(t1, &fin);
  c_mul(t1, t1, t0, s);  // f^(p^6 - 1)
  c_frob(t0, t1, 2, s);
  c_mul(t1, t0, t1, s);  // m = f^((p^6-1)(p^2+1))
  c_pow_x(t0, t1, acc, s);
  c_conj(y0, t1);
  c_mul(y0, t0, y0, s);  // m^(x-1)
  c_pow_x(t0, y0, acc, s);
  c_conj(y1, y0);
  c_mul(y1, t0, y1, s);  // m^((x-1)^2)
  c_pow_x(t0, y1, acc, s);
  c_frob(y2, y1, 1, s);
  c_mul(y2, t0, y2, s);  // y1^(x + p)
  c_pow_x(t0, y2, acc, s);
  c_pow_x(t0, t0, acc, s);  // y2^(x^2)
  c_frob(&y3, y2, 2, s);
  c_mul(&y3, t0, &y3, s);
  c_conj(t0, y2);
  c_mul(&y3, &y3, t0, s);  // y2^(x^2 + p^2 - 1)
  c_mul(t0, t1, t1, s);
  c_mul(t0, t0, t1, s);  // m^3
  c_mul(&y3, &y3, t0, s);
  if (l == 0) w_to_tower(*out, y3);
  __syncthreads();
}

// returns (to every thread) whether f^((p^12 - 1)/r) == 1
__device__ bool c_final_exp_is_one(const fp12_t& f_in, cscratch* s) {
  __shared__ fp12_t r;
  __shared__ uint32_t result;
  c_final_exp(&r, f_in, s);
  if (threadIdx.x == 0) result = fp12_is_one(r) ? 1u : 0u;
  __syncthreads();
  return result != 0;
}

}  // namespace bgv
