// Fp2 = Fp[i] / (i^2 + 1): the field of G2 coordinates and of the tower base.
#pragma once
#include "fp.h"

namespace bgv {

BGV_HD fp2_t fp2_zero() { fp2_t r; fp_set_zero(r.c0); fp_set_zero(r.c1); return r; }
BGV_HD fp2_t fp2_one() { fp2_t r; r.c0 = FP_ONE; fp_set_zero(r.c1); return r; }

BGV_HD bool fp2_is_zero(const fp2_t& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BGV_HD bool fp2_eq(const fp2_t& a, const fp2_t& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BGV_HD bool fp2_is_one(const fp2_t& a) { return fp_eq(a.c0, FP_ONE) && fp_is_zero(a.c1); }

BGV_HD void fp2_select(fp2_t& r, bool c, const fp2_t& a, const fp2_t& b) {
  fp_select(r.c0, c, a.c0, b.c0);
  fp_select(r.c1, c, a.c1, b.c1);
}

// two independent modular operations at once (one asm block, interleaved
// carry chains on the device; fp_asm.h)
BGV_HD void fp_add2(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1) {
#if BGV_ASM_ON
  fpa_add_add(r0, a0, b0, r1, a1, b1);
#else
  fp_add(r0, a0, b0);
  fp_add(r1, a1, b1);
#endif
}
BGV_HD void fp_sub2(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1) {
#if BGV_ASM_ON
  fpa_sub_sub(r0, a0, b0, r1, a1, b1);
#else
  fp_sub(r0, a0, b0);
  fp_sub(r1, a1, b1);
#endif
}
// r0 = a0 + b0, r1 = a1 - b1
BGV_HD void fp_add_sub(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1) {
#if BGV_ASM_ON
  fpa_add_sub(r0, a0, b0, r1, a1, b1);
#else
  fp_add(r0, a0, b0);
  fp_sub(r1, a1, b1);
#endif
}
// r0 = a0 + b0 unreduced (< 2p, product input only), r1 = a1 - b1 mod p
BGV_HD void fp_addnr_sub(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1) {
#if BGV_ASM_ON && BGV_FPMUL28_LAZY
  fpa_addnr_sub(r0, a0, b0, r1, a1, b1);
#else
  fp_add_lazy(r0, a0, b0);
  fp_sub(r1, a1, b1);
#endif
}
BGV_HD void fp_add_lazy2(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1) {
#if BGV_ASM_ON && BGV_FPMUL28_LAZY
  fpa_addnr_addnr(r0, a0, b0, r1, a1, b1);
#else
  fp_add_lazy(r0, a0, b0);
  fp_add_lazy(r1, a1, b1);
#endif
}

// three independent modular additions / subtractions (one asm block)
BGV_HD void fp_add3(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1, fp_t& r2,
                    const fp_t& a2, const fp_t& b2) {
#if BGV_ASM_ON
  fpa_add_add_add(r0, a0, b0, r1, a1, b1, r2, a2, b2);
#else
  fp_add(r0, a0, b0);
  fp_add(r1, a1, b1);
  fp_add(r2, a2, b2);
#endif
}
BGV_HD void fp_sub3(fp_t& r0, const fp_t& a0, const fp_t& b0, fp_t& r1, const fp_t& a1, const fp_t& b1, fp_t& r2,
                    const fp_t& a2, const fp_t& b2) {
#if BGV_ASM_ON
  fpa_sub_sub_sub(r0, a0, b0, r1, a1, b1, r2, a2, b2);
#else
  fp_sub(r0, a0, b0);
  fp_sub(r1, a1, b1);
  fp_sub(r2, a2, b2);
#endif
}

BGV_HD void fp2_add(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp_add2(r.c0, a.c0, b.c0, r.c1, a.c1, b.c1); }
BGV_HD void fp2_sub(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp_sub2(r.c0, a.c0, b.c0, r.c1, a.c1, b.c1); }
BGV_HD void fp2_dbl(fp2_t& r, const fp2_t& a) { fp_add2(r.c0, a.c0, a.c0, r.c1, a.c1, a.c1); }
BGV_HD void fp2_neg(fp2_t& r, const fp2_t& a) {
  const fp_t z = fp_zero();
  fp_sub2(r.c0, z, a.c0, r.c1, z, a.c1);
}
BGV_HD void fp2_conj(fp2_t& r, const fp2_t& a) { r.c0 = a.c0; fp_neg(r.c1, a.c1); }
BGV_HD void fp2_mul3(fp2_t& r, const fp2_t& a) { fp2_t t; fp2_dbl(t, a); fp2_add(r, t, a); }
BGV_HD void fp2_mul4(fp2_t& r, const fp2_t& a) { fp2_t t; fp2_dbl(t, a); fp2_dbl(r, t); }
BGV_HD void fp2_mul8(fp2_t& r, const fp2_t& a) { fp2_t t; fp2_dbl(t, a); fp2_dbl(t, t); fp2_dbl(r, t); }

// The Fp2 product as two sums of products, one Montgomery reduction each
// (fp_mulsum28_digits): c0 = a0 b0 + (2p - a1) b1, c1 = a0 b1 + a1 b0, for
// operands < 2p.  The digit products are those of three Karatsuba products;
// what goes is one unpack / pack / final subtraction and the five Karatsuba
// additions (the leaf is ~1,700 instructions against ~1,950 for three Fp
// leaves and their additions, tools/ubench_fp2.hip).  The result is the
// canonical product, bit-identical to Karatsuba's.
BGV_HD void fp2_mul_sop(fp2_t& r, const fp2_t& a, const fp2_t& b) {
  fp_t na1;  // 2p - a1, no reduction (a1 <= 2p)
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t p2 = (P_MOD.l[i] << 1) | (i ? P_MOD.l[i - 1] >> 31 : 0u);
    na1.l[i] = subb32(p2, a.c1.l[i], br, br);
  }
  uint32_t A0[14], A1[14], N1[14], B0[14], B1[14];
  unpack28<8>(A0, a.c0);
  unpack28<8>(A1, a.c1);
  unpack28<8>(N1, na1);
  unpack28<0>(B0, b.c0);
  unpack28<0>(B1, b.c1);
  fp_t c0, c1;
  fp_mulsum28_digits(c0, A0, B0, N1, B1);
  fp_mulsum28_digits(c1, A0, B1, A1, B0);
  r.c0 = c0;
  r.c1 = c1;
}

// BGV_FP2_LEAF: on the device, every Fp2 product of a unit that calls its
// products (BGV_FPMUL_CALL) is ONE call to this leaf.  Its 48 argument dwords
// exceed the 32 argument VGPRs of the calling convention, so b.c1 travels on
// the stack; the result comes back in v0-v23.
#ifndef BGV_FP2_LEAF
#define BGV_FP2_LEAF 1
#endif
#if defined(__HIPCC__) && BGV_FPMUL_CALL && BGV_FP2_LEAF
typedef uint32_t fp2_vec_t __attribute__((ext_vector_type(24)));
static __device__ __noinline__ fp2_vec_t fp2_mul_leaf(fp_vec_t a0, fp_vec_t a1, fp_vec_t b0, fp_vec_t b1) {
  fp2_t a, b, r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    a.c0.l[i] = a0[i];
    a.c1.l[i] = a1[i];
    b.c0.l[i] = b0[i];
    b.c1.l[i] = b1[i];
  }
  fp2_mul_sop(r, a, b);
  fp2_vec_t v;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    v[i] = r.c0.l[i];
    v[NL + i] = r.c1.l[i];
  }
  return v;
}
#endif

BGV_HD void fp2_mul_body(fp2_t& r, const fp2_t& a, const fp2_t& b) {
#if defined(__HIP_DEVICE_COMPILE__) && BGV_FPMUL_CALL && BGV_FP2_LEAF
#ifdef BGV_COUNT_OPS
  bgv_fpmul_count += 3;
#endif
  fp_vec_t a0, a1, b0, b1;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    a0[i] = a.c0.l[i];
    a1[i] = a.c1.l[i];
    b0[i] = b.c0.l[i];
    b1[i] = b.c1.l[i];
  }
  const fp2_vec_t v = fp2_mul_leaf(a0, a1, b0, b1);
#pragma unroll
  for (int i = 0; i < NL; i++) {
    r.c0.l[i] = v[i];
    r.c1.l[i] = v[NL + i];
  }
#else
  // Karatsuba: 3 Fp products
  fp_t t0, t1, t2, t3;
  fp_mul(t0, a.c0, b.c0);
  fp_mul(t1, a.c1, b.c1);
  fp_add_lazy2(t2, a.c0, a.c1, t3, b.c0, b.c1);  // < 2p, product inputs only
  fp_mul(t2, t2, t3);
  fp_sub2(r.c0, t0, t1, t2, t2, t0);
  fp_sub(r.c1, t2, t1);
#endif
}

BGV_NI2 void fp2_mul(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp2_mul_body(r, a, b); }

// force-inlined copy for call sites that want the products scheduled
// together with their neighbours (Fp6 multiplications, see fp12.h)
BGV_HD void fp2_mul_inl(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp2_mul_body(r, a, b); }

// complex squaring: 2 Fp products
BGV_NI2 void fp2_sqr(fp2_t& r, const fp2_t& a) {
  fp_t t0, t1, t2;
  fp_addnr_sub(t0, a.c0, a.c1, t1, a.c0, a.c1);  // t0 < 2p, product input only
  fp_mul(t2, a.c0, a.c1);
  fp_mul(r.c0, t0, t1);
  fp_dbl(r.c1, t2);
}

BGV_NI2 void fp2_mul_fp(fp2_t& r, const fp2_t& a, const fp_t& b) { fp_mul(r.c0, a.c0, b); fp_mul(r.c1, a.c1, b); }

// multiply by the tower non-residue xi = 1 + i
BGV_HD void fp2_mul_xi(fp2_t& r, const fp2_t& a) {
  fp_t t0, t1;
  fp_add_sub(t1, a.c0, a.c1, t0, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}

// norm a0^2 + a1^2 in Fp
BGV_HD void fp2_norm(fp_t& r, const fp2_t& a) {
  fp_t t0, t1;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(r, t0, t1);
}

BGV_NI void fp2_inv(fp2_t& r, const fp2_t& a) {
  fp_t n, t;
  fp2_norm(n, a);
  fp_inv(n, n);
  fp_mul(r.c0, a.c0, n);
  fp_mul(t, a.c1, n);
  fp_neg(r.c1, t);
}

// RFC 9380 sgn0 for Fp2
BGV_HD uint32_t fp2_sgn0(const fp2_t& a) {
  const uint32_t s0 = fp_parity(a.c0);
  const uint32_t z0 = fp_is_zero(a.c0) ? 1u : 0u;
  const uint32_t s1 = fp_parity(a.c1);
  return s0 | (z0 & s1);
}

// ZCash serialization sign: c1 decides unless zero, then c0.  Both signs are
// computed and selected: no data-dependent return.  gfx950 miscompiled the
// early-return form of this choice under a divergent exec mask on the
// digit-form branch (overlapping spill reloads of the two arms: one signature
// in 66,640 decoded to -y); test_gpu_decode_mixed.py puts
// y.c1 = 0 and y.c0 = 0 lanes beside ordinary ones in one wave.
BGV_HD bool fp2_lex_largest(const fp2_t& a) {
  const bool z1 = fp_is_zero(a.c1);
  const bool l1 = fp_lex_largest(a.c1), l0 = fp_lex_largest(a.c0);
  return z1 ? l0 : l1;
}

// Square root in Fp2 through two Fp exponentiations (p = 3 mod 4):
//   d = sqrt(a0^2 + a1^2)            (exists iff a is a square in Fp2)
//   t = (a0 + d) / 2,  s = t^((p-3)/4)
//   s^2 t == 1 :  x = s t + (a1 s / 2) i
//   otherwise  :  x = (a1 s / 2) - (s t) i      (then -t is the square)
// fp2_sqrt_tail is the second half, for a1 != 0 and a known root d of the
// norm (either sign works: the two choices of t differ by a non-square factor).
BGV_NI void fp2_sqrt_tail(fp2_t& r, const fp2_t& a, const fp_t& d) {
  fp_t t, s, st, s2t, as;
  fp_add(t, a.c0, d);
  fp_half(t, t);
  fp_pow_sqrt_tail(s, t);
  fp_mul(st, s, t);
  fp_mul(s2t, st, s);
  fp_mul(as, a.c1, s);
  fp_half(as, as);
  if (fp_eq(s2t, FP_ONE)) {
    r.c0 = st;
    r.c1 = as;
  } else {
    r.c0 = as;
    fp_neg(r.c1, st);
  }
}

// a1 == 0 is handled directly in Fp.  Returns false iff a is a non-square.
// One exit and no data-dependent return (the arms diverge inside a wave when
// y.c1 = 0 lanes sit beside ordinary ones; see fp2_lex_largest).
BGV_NI bool fp2_sqrt(fp2_t& r, const fp2_t& a) {
  bool ok = true;
  if (fp_is_zero(a.c1)) {
    // s = a0^((p+1)/4) squares to a0 a0^((p-1)/2) = +-a0.  For a non-residue
    // a0, -a0 is a square (-1 is a non-residue) and its root
    // (-a0)^((p+1)/4) = -s ((p+1)/4 is odd): x = -s i
    fp_t s, ns, z;
    const bool re = fp_sqrt(s, a.c0);
    fp_neg(ns, s);
    fp_set_zero(z);
    fp_select(r.c0, re, s, z);
    fp_select(r.c1, re, z, ns);
  } else {
    fp_t n, d;
    fp2_norm(n, a);
    ok = fp_sqrt(d, n);
    if (ok) fp2_sqrt_tail(r, a, d);
    else r = a;
  }
  return ok;
}

// a is a square in Fp2 iff its norm is a square in Fp
BGV_NI bool fp2_is_square(const fp2_t& a) {
  fp_t n, l;
  fp2_norm(n, a);
  if (fp_is_zero(n)) return true;
  fp_pow(l, n, EXP_P_MINUS_1_DIV_2);
  return fp_eq(l, FP_ONE);
}

}  // namespace bgv
