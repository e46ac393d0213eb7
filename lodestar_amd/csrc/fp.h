// Fp: the BLS12-381 base field, 381-bit prime p, on the CDNA4 VALU.
//
// Representation: 12 x u32 limbs, little-endian, Montgomery form with
// R = 2^384.  All values are kept fully reduced in [0, p).  Products are
// formed with 32x32->64 multiply-adds (v_mad_u64_u32 on gfx950); the field is
// an integer-VALU workload, not a dense contraction, so no MFMA is involved.
//
// Re-creates the base-field layer of blst (third-party, reached through
// @chainsafe/blst from packages/beacon-node/src/chain/bls/maybeBatch.ts:18-37);
// this is a from-scratch design for 64-wide wavefronts, one element per lane.
#pragma once
#include "bls_types.h"
#include "bls_consts.h"

namespace bgv {

BGV_HD void fp_set_zero(fp_t& r) {
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = 0;
}

BGV_HD fp_t fp_zero() { fp_t r; fp_set_zero(r); return r; }
BGV_HD fp_t fp_one() { return FP_ONE; }

BGV_HD bool fp_is_zero(const fp_t& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) acc |= a.l[i];
  return acc == 0;
}

BGV_HD bool fp_eq(const fp_t& a, const fp_t& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}

// r = c ? a : b  (branch-free, keeps lanes converged)
BGV_HD void fp_select(fp_t& r, bool c, const fp_t& a, const fp_t& b) {
  const uint32_t m = 0u - (uint32_t)c;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (a.l[i] & m) | (b.l[i] & ~m);
}

// r = a - p if a >= p  (a < 2p)
BGV_HD void fp_reduce_once(fp_t& r, const fp_t& a) {
  uint32_t t[NL];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t d = (uint64_t)a.l[i] - P_MOD.l[i] - borrow;
    t[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  // borrow == 1  <=>  a < p  -> keep a
  const uint32_t m = 0u - borrow;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (a.l[i] & m) | (t[i] & ~m);
}

BGV_HD void fp_add(fp_t& r, const fp_t& a, const fp_t& b) {
  fp_t s;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t t = (uint64_t)a.l[i] + b.l[i] + carry;
    s.l[i] = (uint32_t)t;
    carry = (uint32_t)(t >> 32);
  }
  // p < 2^381, so a + b < 2^382 never carries out of 12 limbs
  fp_reduce_once(r, s);
}

BGV_HD void fp_dbl(fp_t& r, const fp_t& a) { fp_add(r, a, a); }

BGV_HD void fp_sub(fp_t& r, const fp_t& a, const fp_t& b) {
  uint32_t t[NL];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t d = (uint64_t)a.l[i] - b.l[i] - borrow;
    t[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
  // if a < b add p back
  const uint32_t m = 0u - borrow;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t s = (uint64_t)t[i] + (P_MOD.l[i] & m) + carry;
    r.l[i] = (uint32_t)s;
    carry = (uint32_t)(s >> 32);
  }
}

BGV_HD void fp_neg(fp_t& r, const fp_t& a) {
  fp_t z;
  fp_set_zero(z);
  fp_sub(r, z, a);
}

// Montgomery product r = a * b / R mod p.
// Operand-scanning CIOS with the "spare top bit" shortcut: p's top limb is
// < 2^29, so the running sum never needs a 13th/14th word (t < 2p throughout).
#ifdef BGV_COUNT_OPS
extern unsigned long long bgv_fpmul_count;  // host op-count build only (tools/opcount.cpp)
#endif
BGV_HD void fp_mul28(fp_t& r, const fp_t& a, const fp_t& b);
BGV_HD void fp_mul32(fp_t& r, const fp_t& a, const fp_t& b);
#ifndef BGV_FPMUL28
#define BGV_FPMUL28 1
#endif
BGV_HD void fp_mul(fp_t& r, const fp_t& a, const fp_t& b) {
#ifdef BGV_COUNT_OPS
  bgv_fpmul_count++;
#endif
#if BGV_FPMUL28
  fp_mul28(r, a, b);
#else
  fp_mul32(r, a, b);
#endif
}

// 12 x 32-bit CIOS (operand scanning)
BGV_HD void fp_mul32(fp_t& r, const fp_t& a, const fp_t& b) {
  uint32_t t[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t bi = b.l[i];
    // t += a * b_i ; first word separately to derive m
    uint64_t s = (uint64_t)a.l[0] * bi + t[0];
    uint32_t A = (uint32_t)(s >> 32);
    const uint32_t t0 = (uint32_t)s;
    const uint32_t m = t0 * P_INV32;
    uint64_t c = (uint64_t)m * P_MOD.l[0] + t0;
    uint32_t C = (uint32_t)(c >> 32);
#pragma unroll
    for (int j = 1; j < NL; j++) {
      s = (uint64_t)a.l[j] * bi + t[j] + A;
      A = (uint32_t)(s >> 32);
      c = (uint64_t)m * P_MOD.l[j] + (uint32_t)s + C;
      C = (uint32_t)(c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    t[NL - 1] = A + C;
  }
  fp_t s;
#pragma unroll
  for (int i = 0; i < NL; i++) s.l[i] = t[i];
  fp_reduce_once(r, s);
}

// ---- product-scanning variant on 28-bit digits -------------------------
// The 12 x 32-bit CIOS above keeps every partial product inside a carry
// chain, so hipcc spends ~1,000 v_mov / v_lshl_add_u64 per product building
// 64-bit addends.  Here both operands are split into 14 digits of 28 bits;
// a digit product is < 2^56, so every column of the schoolbook and of the
// Montgomery reduction accumulates in a 64-bit register with one
// v_mad_u64_u32 per digit pair and no carries until the end (27
// independent columns: high ILP).  The representation outside stays
// 12 x 32-bit Montgomery with R = 2^384: `a` enters shifted by 8 bits, so the
// 2^-392 of the 28-bit reduction yields a*b*2^-384.  Output < 2p, then one
// conditional subtraction.
BGV_CONST uint32_t P28[14] = {0xfffaaabu, 0xfefffffu, 0x3ffffb9u, 0xfffeb15u, 0x6241eabu, 0xa0f6b0fu, 0xf6730d2u,
                              0xf38512bu, 0x4774b84u, 0x4bacd76u, 0xba7b643u, 0xe69a4b1u, 0x1ea397fu, 0x001a011u};
constexpr uint32_t P28_INV = 0xffcfffdu;  // -p^-1 mod 2^28
constexpr uint32_t M28 = 0x0fffffffu;

// digit k of (a << shift): bits [28k - shift, 28k - shift + 28) of a
template <int SHIFT>
BGV_HD void unpack28(uint32_t d[14], const fp_t& a) {
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int pos = 28 * k - SHIFT;
    uint32_t v;
    if (pos < 0) {
      v = a.l[0] << (-pos);
    } else {
      const int w = pos >> 5, sh = pos & 31;
      const uint32_t lo = w < NL ? a.l[w] : 0u;
      const uint32_t hi = (w + 1) < NL ? a.l[w + 1] : 0u;
      v = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    }
    d[k] = v & M28;
  }
}

BGV_HD void pack28(fp_t& r, const uint32_t d[14]) {
#pragma unroll
  for (int m = 0; m < NL; m++) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 14; k++) {
      const int lo_bit = 28 * k, rel = lo_bit - 32 * m;  // digit k starts at bit rel of limb m
      if (rel >= 32 || rel <= -28) continue;
      v |= rel >= 0 ? (d[k] << rel) : (d[k] >> (-rel));
    }
    r.l[m] = v;
  }
}

BGV_HD void fp_mul28(fp_t& r, const fp_t& a, const fp_t& b) {
  uint32_t A[14], B[14];
  unpack28<8>(A, a);
  unpack28<0>(B, b);
  uint64_t acc[28];
#pragma unroll
  for (int k = 0; k < 28; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++)
#pragma unroll
    for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)A[i] * B[j];
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t m = ((uint32_t)acc[i] * P28_INV) & M28;
#pragma unroll
    for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += acc[i] >> 28;
  }
  uint32_t d[14];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const uint64_t v = acc[14 + k] + c;
    d[k] = (uint32_t)v & M28;
    c = v >> 28;
  }
  fp_t t;
  pack28(t, d);
  fp_reduce_once(r, t);
}

BGV_HD void fp_sqr(fp_t& r, const fp_t& a) { fp_mul(r, a, a); }

// small multiples by repeated doubling/addition
BGV_HD void fp_mul3(fp_t& r, const fp_t& a) { fp_t t; fp_add(t, a, a); fp_add(r, t, a); }
BGV_HD void fp_mul4(fp_t& r, const fp_t& a) { fp_t t; fp_add(t, a, a); fp_add(r, t, t); }
BGV_HD void fp_mul8(fp_t& r, const fp_t& a) { fp_t t; fp_add(t, a, a); fp_add(t, t, t); fp_add(r, t, t); }

BGV_HD void fp_half(fp_t& r, const fp_t& a) { fp_mul(r, a, FP_HALF); }

// r = a^e for a fixed public exponent e (12 x u32, plain integer).
// Left-to-right binary over the exponent's bits; the bit test is uniform
// across the wavefront (same constant for every lane), so no divergence.
BGV_NI void fp_pow(fp_t& r, const fp_t& a, const fp_t& e) {
  fp_t acc = FP_ONE;
  bool started = false;
  for (int i = NL - 1; i >= 0; i--) {
    const uint32_t w = e.l[i];
    for (int b = 31; b >= 0; b--) {
      if (started) fp_sqr(acc, acc);
      if ((w >> b) & 1) {
        if (started) fp_mul(acc, acc, a);
        else { acc = a; started = true; }
      }
    }
  }
  r = acc;
}

BGV_HD void fp_inv(fp_t& r, const fp_t& a) { fp_pow(r, a, EXP_P_MINUS_2); }

// candidate square root a^((p+1)/4); returns true iff it squares back to a
BGV_HD bool fp_sqrt(fp_t& r, const fp_t& a) {
  fp_t s, chk;
  fp_pow(s, a, EXP_P_PLUS_1_DIV_4);
  fp_sqr(chk, s);
  r = s;
  return fp_eq(chk, a);
}

// ---- conversions --------------------------------------------------------

BGV_HD void fp_to_mont(fp_t& r, const fp_t& a) { fp_mul(r, a, R2_MOD); }

BGV_HD void fp_from_mont(fp_t& r, const fp_t& a) {
  fp_t one;
  fp_set_zero(one);
  one.l[0] = 1;
  fp_mul(r, a, one);
}

// plain-integer comparison a < p
BGV_HD bool fp_plain_lt_p(const fp_t& a) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t d = (uint64_t)a.l[i] - P_MOD.l[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow != 0;
}

// plain-integer comparison a > (p-1)/2 (ZCash "lexicographically largest")
BGV_HD bool fp_plain_gt_half(const fp_t& a) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint64_t d = (uint64_t)P_HALF.l[i] - a.l[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  return borrow != 0;  // (p-1)/2 - a < 0
}

// lexicographic sign of a Montgomery-form element
BGV_HD bool fp_lex_largest(const fp_t& a) {
  fp_t t;
  fp_from_mont(t, a);
  return fp_plain_gt_half(t);
}

// RFC 9380 sgn0 (parity) of a Montgomery-form element
BGV_HD uint32_t fp_parity(const fp_t& a) {
  fp_t t;
  fp_from_mont(t, a);
  return t.l[0] & 1u;
}

// 48 big-endian bytes -> plain limbs (no reduction, no range check)
BGV_HD void fp_from_be48(fp_t& r, const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}

BGV_HD void fp_to_be48(uint8_t* b, const fp_t& a) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    uint8_t* q = b + 44 - 4 * i;
    const uint32_t w = a.l[i];
    q[0] = (uint8_t)(w >> 24); q[1] = (uint8_t)(w >> 16); q[2] = (uint8_t)(w >> 8); q[3] = (uint8_t)w;
  }
}

}  // namespace bgv
