// Cooperative Miller loop: SIX lanes per pair, state in LDS.
//
// The one-lane-per-pair loop (pairing.h) keeps f (576 B), T and the line in
// per-lane scratch and moves every Fp2 operand through it on each call:
// ~16 KB of scratch traffic per lane per iteration, which at 100k resident
// lanes is served from beyond L2 (rocprofv3: ~130 GB FETCH+WRITE per launch).
// Here lane k of a 6-lane group owns coefficient k of
//   f = sum_k f_k w^k  in  Fp12 = Fp2[w] / (w^6 - xi),  xi = 1 + i
// (tower slot of w^k: 0 c0.c0, 1 c1.c0, 2 c0.c1, 3 c1.c1, 4 c0.c2, 5 c1.c2),
// and per iteration the group runs:
//   S   f^2 by the symmetric schoolbook, 4 products per lane   4 Fp2 mul
//   D1  doubling-step products (5 lanes)                       1 Fp2 mul
//   D2  doubling-step products and the line (6 lanes)           1 Fp2 mul
//   L   f * (a0 + a1 w^2 + b1 w^3), 3 products per lane        3 Fp2 mul
// plus the addition-step rounds on the 5 set bits of |x|.  Every product
// goes through ONE non-inlined routine, coop_prod(a, b, out) on LDS
// pointers, so the kernel holds a single copy of the Fp2 multiplication and
// no operand ever travels through scratch; operands that are computed (sums,
// differences) are staged in the lane's own LDS slot first.  Formulas are
// those of pairing.h (miller_dbl_step / miller_add_step), so f is
// bit-identical to miller_loop().  A 64-lane workgroup is one wave;
// __syncthreads() orders the LDS hand-offs between rounds.
#pragma once
#include "pairing.h"

namespace bgv {

// Layouts (template parameters SUB, HALF; the launcher picks one by batch
// size, bgv_kernels.hip):
//   SUB = 3: every coefficient lane k is three sub-lanes q, one per Karatsuba
//     Fp product of each Fp2 product (coop_prod_sub), so a product round
//     costs the latency of ONE Fp product instead of three;
//   HALF = 2 (with SUB = 3): every coefficient lane is also split in two
//     halves h that share the squaring's four products and the line
//     multiplication's three (2 + 2 and 2 + 1 per half), so those steps take
//     2 product rounds instead of 4 and 3;
//   <1, 1> = 6 lanes per pair (10 pairs per wave), <3, 1> = 18 (3 per wave),
//   <3, 2> = 36 (one pair per wave).
template <int SUB, int HALF> struct coop_cfg {
  static_assert((SUB == 1 && HALF == 1) || (SUB == 3 && (HALF == 1 || HALF == 2)), "coop layout");
  static constexpr int LANES = 6 * SUB * HALF;  // lanes per pair
  static constexpr int GROUPS = 64 / LANES;     // pairs per 64-lane workgroup
};
constexpr int COOP_LANES = 6;

template <int SUB, int HALF> struct coop_grp_t {
  fp2_t f[6];     // w-basis coefficients of the accumulator
  fp2_t T[3];     // X, Y, Z (homogeneous projective)
  fp2_t Q[2];     // affine Q (addition steps)
  fp2_t px, py;   // P coordinates as Fp2 (c1 = 0)
  fp2_t line[3];  // a0, a1, b1
  fp2_t r[8];     // per-round products
  fp2_t a[6];     // per-lane staged operand
  // layout-specific exchange slots; zero-length (no LDS) where unused, so
  // the 6-lane layout's 10 groups fit 5 workgroups per CU
  fp_t P[SUB == 3 ? 6 * HALF : 0][3];  // sub-lane Fp products of coefficient lane (k, h)
  fp2_t hs[HALF == 2 ? 6 : 0][2];      // per-half partial sums
  fp2_t ah[HALF == 2 ? 6 : 0][2];      // per-half staged products
};

// f^2 by the symmetric schoolbook in the w-basis: lane k sums 4 products
// f_i f_j (i + j = k mod 6), doubled for i != j, times xi when i + j >= 6; a
// 4th "product" with weight 0 pads the odd lanes so every lane runs the same
// code.  (The tower's complex/Karatsuba squaring needs only 2 products per
// lane, but its per-lane operand sums and divergent recombination cost as
// much on the SIMT lanes as the 2 products saved: measured slower, r01.)
struct sq_term {
  uint8_t i, j, dbl, xi, use;
};
BGV_CONST sq_term SQ_TAB[6][4] = {
    {{0, 0, 0, 0, 1}, {3, 3, 0, 1, 1}, {1, 5, 1, 1, 1}, {2, 4, 1, 1, 1}},
    {{0, 1, 1, 0, 1}, {2, 5, 1, 1, 1}, {3, 4, 1, 1, 1}, {0, 0, 0, 0, 0}},
    {{0, 2, 1, 0, 1}, {1, 1, 0, 0, 1}, {3, 5, 1, 1, 1}, {4, 4, 0, 1, 1}},
    {{0, 3, 1, 0, 1}, {1, 2, 1, 0, 1}, {4, 5, 1, 1, 1}, {0, 0, 0, 0, 0}},
    {{0, 4, 1, 0, 1}, {1, 3, 1, 0, 1}, {2, 2, 0, 0, 1}, {5, 5, 0, 1, 1}},
    {{0, 5, 1, 0, 1}, {1, 4, 1, 0, 1}, {2, 3, 1, 0, 1}, {0, 0, 0, 0, 0}},
};

BGV_HD void fp_half_shift(fp_t& r, const fp_t& a) { fp_half(r, a); }

__device__ __forceinline__ void fp2_half(fp2_t& r, const fp2_t& a) {
  fp_half_shift(r.c0, a.c0);
  fp_half_shift(r.c1, a.c1);
}

// *out = *a * *b  (LDS operands; the one Fp2 multiplication of the kernel)
__device__ __noinline__ void coop_prod(const fp2_t* a, const fp2_t* b, fp2_t* out) {
  const fp2_t x = *a, y = *b;
  fp2_t r;
  fp2_mul_inl(r, x, y);
  *out = r;
}

// LDS hand-off between lanes of one wave (every user is a one-wave
// workgroup): BGV_COOP_SYNC 0 also waits for the wave's LDS writes
#ifndef BGV_COOP_SYNC
#define BGV_COOP_SYNC 1  // r02: cg doubling 7.63 -> 7.36 us, k_hash_clear_coop 1,473 -> 1,448 us, k_miller_coop 1,347 -> 1,325 us (C2 shape)
#endif
#if BGV_COOP_SYNC
// a wave's LDS instructions execute in issue order, so a lane's read after
// another lane's write in the same wave sees it: only the compiler must not
// move LDS accesses across the exchange point
__device__ __forceinline__ void coop_wave_sync() { __builtin_amdgcn_wave_barrier(); __asm__ volatile("" ::: "memory"); }
#else
__device__ __forceinline__ void coop_wave_sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
#endif

// *out = *a * *b over the three sub-lanes q of lane k: q0 a0 b0, q1 a1 b1,
// q2 (a0 + a1)(b0 + b1) (one leaf call on every lane), then q0 / q1 form
// c0 = P0 - P1 / c1 = P2 - P0 - P1.  All three sub-lanes of k call it
// together (the branch conditions around every call depend on k only).
#ifndef BGV_CPROD_ADDR
#define BGV_CPROD_ADDR 1  // operands by address + a masked lazy sum, no divergent 3-way branch
#endif
__device__ __forceinline__ void coop_prod_sub(fp_t* P, uint32_t q, const fp2_t* a, const fp2_t* b, fp2_t* out) {
  fp_t u, v;
#if BGV_CPROD_ADDR
  {
    // sub-lane q: component q (q < 2) or c0 + c1 (q = 2: c1 masked in; a lazy
    // sum of x and 0 is x)
    const uint32_t m = q == 2 ? ~0u : 0u;
    const fp_t xa = *(q == 1 ? &a->c1 : &a->c0), xb = *(q == 1 ? &b->c1 : &b->c0);
    fp_t ma, mb;
#pragma unroll
    for (int k = 0; k < NL; k++) {
      ma.l[k] = a->c1.l[k] & m;
      mb.l[k] = b->c1.l[k] & m;
    }
    fp_add_lazy2(u, xa, ma, v, xb, mb);  // < 2p, product inputs only
  }
#else
  if (q == 0) {
    u = a->c0;
    v = b->c0;
  } else if (q == 1) {
    u = a->c1;
    v = b->c1;
  } else {
    fp_add_lazy(u, a->c0, a->c1);  // < 2p, product inputs only
    fp_add_lazy(v, b->c0, b->c1);
  }
#endif
  fp_t r;
  fp_mul(r, u, v);
  P[q] = r;
  coop_wave_sync();
  if (q < 2) {  // one dual add/sub on both lanes (no divergent branches), lane 1 finishes c1
    fp_t t, w;
    fp_add_sub(w, P[0], P[1], t, P[0], P[1]);
    if (q == 1) fp_sub(t, P[2], w);
    if (q == 0) out->c0 = t;
    else out->c1 = t;
  }
  coop_wave_sync();
}

// one Fp2 product of coefficient lane (k, h): over its three sub-lanes (SUB = 3) or alone
template <int SUB, int HALF>
__device__ __forceinline__ void cprod(coop_grp_t<SUB, HALF>& g, uint32_t k, uint32_t h, uint32_t q, const fp2_t* a,
                                      const fp2_t* b, fp2_t* out) {
  if constexpr (SUB == 3) coop_prod_sub(g.P[k * HALF + h], q, a, b, out);
  else coop_prod(a, b, out);
}
#define COOP_PROD(pa, pb, out) cprod<SUB, HALF>(g, k, h, q, (pa), (pb), (out))

// lanes 0..5: g.r[k] <- c_k of f * (a0 + a1 w^2 + b1 w^3); then f <- that
template <int SUB, int HALF>
__device__ __forceinline__ void coop_line_round(coop_grp_t<SUB, HALF>& g, uint32_t k, uint32_t h, uint32_t q, bool active) {
  fp2_t acc;
  if constexpr (HALF == 2) {
  // half 0: f_k a0 and the w^2 term; half 1: the w^3 term (same sum order)
  if (active) {
    // both halves run two product calls (half 1's second is a dummy into its
    // own slot), so the wave pays two product latencies, not 2 + 1 in turn
    const fp2_t* pa1 = h == 0 ? &g.f[k] : &g.f[(k + 3) % 6];
    const fp2_t* pb1 = h == 0 ? &g.line[0] : &g.line[2];
    COOP_PROD(pa1, pb1, h == 0 ? &g.r[k] : &g.ah[k][1]);
    COOP_PROD(h == 0 ? &g.f[(k + 4) % 6] : pa1, h == 0 ? &g.line[1] : pb1, h == 0 ? &g.ah[k][0] : &g.a[k]);
    if (h == 0) {
      acc = g.r[k];
      fp2_t t = g.ah[k][0];
      if (k < 2) fp2_mul_xi(t, t);
      fp2_add(acc, acc, t);
    } else {
      acc = g.ah[k][1];
      if (k < 3) fp2_mul_xi(acc, acc);
    }
    g.hs[k][h] = acc;
    coop_wave_sync();
    fp2_add(acc, g.hs[k][0], g.hs[k][1]);
  }
  __syncthreads();
  if (active) g.f[k] = acc;
  __syncthreads();
  return;
  }
  if (active) {
    COOP_PROD(&g.f[k], &g.line[0], &g.r[k]);
    acc = g.r[k];
#pragma unroll 1
    for (uint32_t s = 0; s < 2; s++) {
      const uint32_t sh = s ? 3u : 2u;  // w^2 (a1) and w^3 (b1)
      COOP_PROD(&g.f[(k + 6 - sh) % 6], &g.line[1 + s], &g.a[k]);
      fp2_t t = g.a[k];
      if (k < sh) fp2_mul_xi(t, t);
      fp2_add(acc, acc, t);
    }
  }
  __syncthreads();
  if (active) g.f[k] = acc;
  __syncthreads();
}

// Miller loop of the pair held in g (T := Q, P in px/py) by lanes k = 0..5.
// Every lane of the workgroup calls it (barriers inside); lanes outside a
// pair, or of a skipped pair, pass active = false.
template <int SUB, int HALF>
__device__ void coop_miller(coop_grp_t<SUB, HALF>& g, uint32_t k, uint32_t h, uint32_t q, bool active) {
  for (int b = 62; b >= 0; b--) {
    // ---- S: f <- f^2 (not on the first iteration: f = 1)
    if (b != 62) {
      fp2_t acc = fp2_zero();
      if (active) {
        if constexpr (HALF == 2) {
        // half h: products 2h, 2h + 1 of lane k; (t0 + t1) + (t2 + t3)
#pragma unroll 1
        for (int p = 2 * (int)h; p < 2 * (int)h + 2; p++) {
          const sq_term e = SQ_TAB[k][p];
          COOP_PROD(&g.f[e.i], &g.f[e.j], &g.ah[k][h]);
          fp2_t t = g.ah[k][h];
          if (e.dbl) fp2_dbl(t, t);
          if (e.xi) fp2_mul_xi(t, t);
          if (e.use) fp2_add(acc, acc, t);
        }
        g.hs[k][h] = acc;
        coop_wave_sync();
        fp2_add(acc, g.hs[k][0], g.hs[k][1]);
        } else {
#pragma unroll 1
        for (int p = 0; p < 4; p++) {
          const sq_term e = SQ_TAB[k][p];
          COOP_PROD(&g.f[e.i], &g.f[e.j], &g.a[k]);
          fp2_t t = g.a[k];
          if (e.dbl) fp2_dbl(t, t);
          if (e.xi) fp2_mul_xi(t, t);
          if (e.use) fp2_add(acc, acc, t);
        }
        }
      }
      __syncthreads();
      if (active) g.f[k] = acc;
      __syncthreads();
    }
    // ---- D1: products of the doubling step that only need T
    //   k0: X*Y  k1: Y^2  k2: Z^2  k3: (Y+Z)^2  k4: X^2      -> r[k]
    if (active && k < 5) {
      const fp2_t* pa = &g.T[0];
      const fp2_t* pb = &g.T[1];
      if (k == 1) pa = &g.T[1];
      else if (k == 2) pa = pb = &g.T[2];
      else if (k == 3) {
        fp2_add(g.a[k], g.T[1], g.T[2]);
        pa = pb = &g.a[k];
      } else if (k == 4) pb = &g.T[0];
      COOP_PROD(pa, pb, &g.r[k]);
    }
    __syncthreads();
    // ---- D2: the rest of miller_dbl_step (same formulas):
    //   A = XY/2, B = Y^2, C = Z^2, E = 3b'C, F = 3E, H = (Y+Z)^2 - B - C
    //   a0 = E - B, a1 = 3X^2 xP, b1 = -H yP
    //   X' = A (B - F) = (XY (B - F)) / 2, Y' = ((B + F)/2)^2 - 3E^2, Z' = B H
    //   k0: XY (B-F)  k1: E^2  k2: ((B+F)/2)^2  k3: B H  k4: 3X^2 xP  k5: H yP
    fp2_t mine;
    if (active) {
      fp2_t E, F, H;
      const fp2_t B = g.r[1], C = g.r[2];
      fp2_mul_xi(E, C);  // 3b' C = 12 (1 + i) C by additions
      fp2_mul4(E, E);
      fp2_mul3(E, E);
      fp2_mul3(F, E);
      fp2_add(H, B, C);
      fp2_sub(H, g.r[3], H);
      const fp2_t* pa = &g.a[k];
      const fp2_t* pb = &g.a[k];
      if (k == 0) { fp2_sub(g.a[k], B, F); pb = &g.r[0]; }
      else if (k == 1) g.a[k] = E;
      else if (k == 2) { fp2_t t; fp2_add(t, B, F); fp2_half(g.a[k], t); }
      else if (k == 3) { g.a[k] = H; pb = &g.r[1]; }
      else if (k == 4) { fp2_mul3(g.a[k], g.r[4]); pb = &g.px; }
      else { g.a[k] = H; pb = &g.py; }
      if (k == 1) fp2_sub(mine, E, B);  // a0
      __syncthreads();                   // r[0..4] fully read before r[5..] / r[k] writes
      COOP_PROD(pa, pb, &g.r[k == 0 ? 0 : k + 2]);
    } else {
      __syncthreads();
    }
    __syncthreads();
    // r0 = XY(B-F), r3 = E^2, r4 = ((B+F)/2)^2, r5 = B H, r6 = 3X^2 xP, r7 = H yP
    if (active) {
      if (k == 0) fp2_half(g.T[0], g.r[0]);
      else if (k == 1) g.line[0] = mine;
      else if (k == 2) { fp2_t t; fp2_mul3(t, g.r[3]); fp2_sub(g.T[1], g.r[4], t); }
      else if (k == 3) g.T[2] = g.r[5];
      else if (k == 4) g.line[1] = g.r[6];
      else fp2_neg(g.line[2], g.r[7]);
    }
    __syncthreads();
    // ---- L: f <- f * line (first iteration: f = line)
    if (b == 62) {
      if (active) {
        fp2_t v = fp2_zero();
        if (k == 0) v = g.line[0];
        else if (k == 2) v = g.line[1];
        else if (k == 3) v = g.line[2];
        g.f[k] = v;
      }
      __syncthreads();
    } else {
      coop_line_round(g, k, h, q, active);
    }
    if (!((BLS_X_ABS >> b) & 1ull)) continue;
    // ---- addition step (miller_add_step)
    //   R1  k0: yQ Z  k1: xQ Z                               -> r0, r1
    if (active && k < 2) COOP_PROD(k ? &g.Q[0] : &g.Q[1], &g.T[2], &g.r[k]);
    __syncthreads();
    //   th = Y - yQ Z (-> r6), la = X - xQ Z (-> r7)
    //   R2  k0: th xQ  k1: la yQ  k2: th xP  k3: la yP  k4: th^2 = C  k5: la^2 = D
    if (active) {
      fp2_t th, la;
      fp2_sub(th, g.T[1], g.r[0]);
      fp2_sub(la, g.T[0], g.r[1]);
      g.a[k] = (k & 1) ? la : th;
      const fp2_t* pb = &g.a[k];
      if (k == 0) pb = &g.Q[0];
      else if (k == 1) pb = &g.Q[1];
      else if (k == 2) pb = &g.px;
      else if (k == 3) pb = &g.py;
      __syncthreads();  // r0, r1 read by every lane before r[k] is overwritten
      COOP_PROD(&g.a[k], pb, &g.r[k]);
      if (k == 0) g.r[6] = th;
      if (k == 1) g.r[7] = la;
    } else {
      __syncthreads();
    }
    __syncthreads();
    // line: a0 = th xQ - la yQ, a1 = -th xP, b1 = la yP
    //   R3  k0: E = D la  k1: F = Z C  k2: G = X D            -> a[k] (staged)
    if (active && k < 3) {
      const fp2_t* pa = &g.r[5];
      const fp2_t* pb = &g.r[7];
      if (k == 1) { pa = &g.T[2]; pb = &g.r[4]; }
      else if (k == 2) { pa = &g.T[0]; pb = &g.r[5]; }
      COOP_PROD(pa, pb, &g.a[k]);
    }
    if (active && k == 3) {
      fp2_sub(g.line[0], g.r[0], g.r[1]);
      fp2_neg(g.line[1], g.r[2]);
      g.line[2] = g.r[3];
    }
    __syncthreads();
    //   H = E + F - 2G
    //   R4  k0: X' = la H  k1: th (G - H)  k2: Y E  k3: Z' = Z E   -> r0..r3
    if (active && k < 4) {
      fp2_t Hh;
      const fp2_t Ee = g.a[0], Ff = g.a[1], Gg = g.a[2];
      fp2_add(Hh, Ee, Ff);
      fp2_sub(Hh, Hh, Gg);
      fp2_sub(Hh, Hh, Gg);
      fp2_t opd;
      const fp2_t* pa;
      const fp2_t* pb = &g.r[3 + k];  // placeholder, set below
      if (k == 0) { opd = Hh; pb = &g.r[7]; }
      else if (k == 1) { fp2_sub(opd, Gg, Hh); pb = &g.r[6]; }
      else if (k == 2) { opd = Ee; pb = &g.T[1]; }
      else { opd = Ee; pb = &g.T[2]; }
      __syncthreads();  // a[0..2] read by every lane before being restaged
      g.a[k] = opd;
      pa = &g.a[k];
      COOP_PROD(pa, pb, &g.r[k]);
    } else {
      __syncthreads();
    }
    __syncthreads();
    if (active && k == 0) {
      g.T[0] = g.r[0];
      fp2_sub(g.T[1], g.r[1], g.r[2]);
      g.T[2] = g.r[3];
    }
    __syncthreads();
    coop_line_round(g, k, h, q, active);
  }
  // x < 0: conjugate (negate the odd powers of w)
  if (active && (k & 1)) fp2_neg(g.f[k], g.f[k]);
  __syncthreads();
}

}  // namespace bgv
