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
#ifndef BGV_FPMUL28
#define BGV_FPMUL28 1
#endif
#ifndef BGV_FPMUL28_LAZY
#define BGV_FPMUL28_LAZY BGV_FPMUL28
#endif

// 32-bit carry / borrow steps.  Under clang they are the add/sub-with-carry
// builtins, so a 12-limb chain is v_add_co/v_addc_co (v_sub_co/v_subb_co)
// on gfx950; the 64-bit "d >> 63" form compiled to sign extensions plus a
// hazard NOP per limb.  g++ (host tests) takes the portable form.
BGV_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
#if defined(__clang__)
  unsigned int co;
  const uint32_t s = __builtin_addc(a, b, cin, &co);
  cout = co;
  return s;
#else
  const uint64_t t = (uint64_t)a + b + cin;
  cout = (uint32_t)(t >> 32);
  return (uint32_t)t;
#endif
}
BGV_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
#if defined(__clang__)
  unsigned int bo;
  const uint32_t d = __builtin_subc(a, b, bin, &bo);
  bout = bo;
  return d;
#else
  const uint64_t d = (uint64_t)a - b - bin;
  bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}

BGV_HD void fp_reduce_once(fp_t& r, const fp_t& a) {
  uint32_t t[NL];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) t[i] = subb32(a.l[i], P_MOD.l[i], borrow, borrow);
  // borrow == 1  <=>  a < p  -> keep a
  const uint32_t m = 0u - borrow;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = (a.l[i] & m) | (t[i] & ~m);
}

#ifndef BGV_ASM_ADD
#define BGV_ASM_ADD 1  // device: interleaved-chain inline asm (fp_asm.h)
#endif
#if defined(__HIP_DEVICE_COMPILE__) && BGV_ASM_ADD
#define BGV_ASM_ON 1
#else
#define BGV_ASM_ON 0
#endif
}  // namespace bgv
#include "fp_asm.h"
namespace bgv {

BGV_HD void fp_add(fp_t& r, const fp_t& a, const fp_t& b) {
#if BGV_ASM_ON
  fpa_add(r, a, b);
  return;
#endif
  fp_t s;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) s.l[i] = addc32(a.l[i], b.l[i], carry, carry);
  // p < 2^381, so a + b < 2^382 never carries out of 12 limbs
  fp_reduce_once(r, s);
}

BGV_HD void fp_dbl(fp_t& r, const fp_t& a) { fp_add(r, a, a); }

// Lazy forms, ONLY for operands that go straight into fp_mul: the result is
// < 2p < 2^382 (not reduced).  fp_mul28 accepts inputs < 2^382 (the 8-bit
// pre-shift still fits its 14 x 28-bit digits) and, with both inputs < 2p,
// its Montgomery sum stays below 4p^2 2^8 / 2^392 + p < 1.41 p before the
// final subtraction, so its output is canonical.  The 32-bit CIOS variant
// (BGV_FPMUL28=0) keeps the reduced forms.
BGV_HD void fp_add_lazy(fp_t& r, const fp_t& a, const fp_t& b) {
#if BGV_FPMUL28_LAZY
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = addc32(a.l[i], b.l[i], carry, carry);
#else
  fp_add(r, a, b);
#endif
}

BGV_HD void fp_sub(fp_t& r, const fp_t& a, const fp_t& b) {
#if BGV_ASM_ON
  fpa_sub(r, a, b);
  return;
#endif
  uint32_t t[NL];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) t[i] = subb32(a.l[i], b.l[i], borrow, borrow);
  // if a < b add p back
  const uint32_t m = 0u - borrow;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = addc32(t[i], P_MOD.l[i] & m, carry, carry);
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
// BGV_FPMUL_CALL=1: on the device, every product is a call to ONE non-inlined
// leaf whose operands and result are 12-element vectors, which the AMDGPU
// calling convention keeps in VGPRs (v0-v23 in, v0-v11 out).  By-reference or
// struct arguments would travel through the scratch stack.
#ifndef BGV_FPMUL_CALL
#define BGV_FPMUL_CALL 0
#endif
#if defined(__HIPCC__) && BGV_FPMUL_CALL
typedef uint32_t fp_vec_t __attribute__((ext_vector_type(12)));
static __device__ __noinline__ fp_vec_t fp_mul_leaf(fp_vec_t a, fp_vec_t b);
#endif
BGV_HD void fp_mul(fp_t& r, const fp_t& a, const fp_t& b) {
#ifdef BGV_COUNT_OPS
  bgv_fpmul_count++;
#endif
#if defined(__HIP_DEVICE_COMPILE__) && BGV_FPMUL_CALL
  fp_vec_t va, vb;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    va[i] = a.l[i];
    vb[i] = b.l[i];
  }
  const fp_vec_t vr = fp_mul_leaf(va, vb);
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = vr[i];
#elif BGV_FPMUL28
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

// Sum of two products with ONE Montgomery reduction, on pre-split digits:
// r = (a b + c d) 2^-384 mod p with A = digits(a << 8), C = digits(c << 8),
// B = digits(b), D = digits(d).  Column bound: 28 digit products < 2^60.8 +
// 14 reduction terms < 2^59.8 + carry < 2^62.  Output before the final
// subtraction < (a b + c d) / 2^384 + p, canonical after it whenever
// a b + c d < 2^384 p (e.g. every operand < 2p: 8 p^2 < 2^384 p).  The Fp2
// product below computes each coefficient this way: the same 4 x 196 + 2 x 196
// digit products as three Karatsuba products, with two unpack/pack/final
// subtractions instead of three and no Karatsuba additions.
BGV_HD void fp_mulsum28_digits(fp_t& r, const uint32_t A[14], const uint32_t B[14], const uint32_t C[14], const uint32_t D[14]) {
  uint64_t acc[28];
#pragma unroll
  for (int k = 0; k < 28; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++)
#pragma unroll
    for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)A[i] * B[j] + (uint64_t)C[i] * D[j];
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

// Squaring on the same digits: both operands are a << 4, so the square
// carries the 2^8 of the pre-shift; the 91 cross products are summed once
// against a doubled digit (2 A_j < 2^29), 105 digit products instead of 196.
// Column bound: 7 cross terms < 2^57 + 1 square < 2^56 + 14 reduction terms
// < 2^56 + carry < 2^61.  Inputs < 2^382 (lazy sums) as for fp_mul28; the
// Montgomery sum stays < 1.5 p, so one subtraction leaves it canonical.
BGV_HD void fp_sqr28(fp_t& r, const fp_t& a) {
  uint32_t A[14], D[14];
  unpack28<4>(A, a);
#pragma unroll
  for (int j = 0; j < 14; j++) D[j] = A[j] << 1;
  uint64_t acc[28];
#pragma unroll
  for (int k = 0; k < 28; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    acc[2 * i] += (uint64_t)A[i] * A[i];
#pragma unroll
    for (int j = i + 1; j < 14; j++) acc[i + j] += (uint64_t)A[i] * D[j];
  }
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

#if defined(__HIPCC__) && BGV_FPMUL_CALL
static __device__ __noinline__ fp_vec_t fp_sqr_leaf(fp_vec_t a) {
  fp_t x, r;
#pragma unroll
  for (int i = 0; i < NL; i++) x.l[i] = a[i];
  fp_sqr28(r, x);
  fp_vec_t v;
#pragma unroll
  for (int i = 0; i < NL; i++) v[i] = r.l[i];
  return v;
}

static __device__ __noinline__ fp_vec_t fp_mul_leaf(fp_vec_t a, fp_vec_t b) {
  fp_t x, y, r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    x.l[i] = a[i];
    y.l[i] = b[i];
  }
  fp_mul28(r, x, y);
  fp_vec_t v;
#pragma unroll
  for (int i = 0; i < NL; i++) v[i] = r.l[i];
  return v;
}
#endif

#ifndef BGV_FPSQR
#define BGV_FPSQR 1  // dedicated squaring (fp_sqr28); 0 = fp_mul(a, a)
#endif
BGV_HD void fp_sqr(fp_t& r, const fp_t& a) {
#if BGV_FPSQR && BGV_FPMUL28
#ifdef BGV_COUNT_OPS
  bgv_fpmul_count++;
#endif
#if defined(__HIP_DEVICE_COMPILE__) && BGV_FPMUL_CALL
  fp_vec_t va;
#pragma unroll
  for (int i = 0; i < NL; i++) va[i] = a.l[i];
  const fp_vec_t vr = fp_sqr_leaf(va);
#pragma unroll
  for (int i = 0; i < NL; i++) r.l[i] = vr[i];
#else
  fp_sqr28(r, a);
#endif
#else
  fp_mul(r, a, a);
#endif
}

// small multiples by repeated doubling/addition
BGV_HD void fp_mul3(fp_t& r, const fp_t& a) { fp_t t; fp_add(t, a, a); fp_add(r, t, a); }
BGV_HD void fp_mul4(fp_t& r, const fp_t& a) { fp_t t; fp_add(t, a, a); fp_add(r, t, t); }
BGV_HD void fp_mul8(fp_t& r, const fp_t& a) { fp_t t; fp_add(t, a, a); fp_add(t, t, t); fp_add(r, t, t); }

// a / 2 mod p by a shift: (a + (a odd ? p : 0)) >> 1  (a < p, so a + p < 2^382);
// ~40 VALU instructions instead of a product by 1/2
BGV_HD void fp_half(fp_t& r, const fp_t& a) {
  const uint32_t m = 0u - (a.l[0] & 1u);
  uint32_t t[NL];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) t[i] = addc32(a.l[i], P_MOD.l[i] & m, c, c);
#pragma unroll
  for (int i = 0; i < NL - 1; i++) r.l[i] = (t[i] >> 1) | (t[i + 1] << 31);
  r.l[NL - 1] = t[NL - 1] >> 1;
}

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

// ---- inversion: Bernstein-Yang divsteps ("safegcd"), 30 per round ----------
// Replaces a^(p-2) (381 squarings + ~190 products) with ~27 rounds of 30
// branch-free divsteps on the low limbs plus one 2x2 matrix update of the
// full-width values: ~1/10 of the instructions.  Variable time (the round
// loop stops when g = 0; inputs are public here), capped at the proven
// bound ceil(1101/30) = 37 rounds for 381-bit moduli (Bernstein & Yang 2019,
// thm 11.2).
//   f = p, g = x, d = 0, e = 1 with  d x = f, e x = g (mod p);  each round
//   (f, g) <- M (f, g) / 2^30, (d, e) <- M (d, e) / 2^30 mod p;  at the end
//   g = 0, f = +-1, so x^-1 = +-d.
// Values are 13 signed 30-bit limbs: limbs 0..11 in [0, 2^30), limb 12 signed.
struct s30_t {
  int32_t v[13];
};
constexpr int32_t S30_MASK = (1 << 30) - 1;

BGV_HD void s30_from_fp(s30_t& r, const fp_t& a) {
#pragma unroll
  for (int i = 0; i < 13; i++) {
    const int w = (30 * i) / 32, sh = (30 * i) % 32;
    uint32_t x = a.l[w] >> sh;
    if (sh > 2 && w + 1 < NL) x |= a.l[w + 1] << (32 - sh);
    r.v[i] = (int32_t)(x & S30_MASK);
  }
}

// a must be normalized and in [0, 2^384)
BGV_HD void s30_to_fp(fp_t& r, const s30_t& a) {
#pragma unroll
  for (int w = 0; w < NL; w++) {
    const int i = (32 * w) / 30, sh = (32 * w) % 30;
    uint32_t x = (uint32_t)a.v[i] >> sh;
    x |= (uint32_t)a.v[i + 1] << (30 - sh);  // sh = 2w mod 30 <= 28: two limbs cover a word
    r.l[w] = x;
  }
}

// 30 divsteps on the low limbs: delta, and the transition matrix
// [u v; q r] with 2^30 (f', g') = [u v; q r] (f, g), |u|+|v|, |q|+|r| <= 2^30
BGV_HD void divsteps30(int32_t& delta, uint32_t f, uint32_t g, int32_t& u_, int32_t& v_, int32_t& q_, int32_t& r_) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    const uint32_t godd = 0u - (g & 1u);
    const uint32_t c = (uint32_t)((-delta) >> 31) & godd;  // swap: delta > 0 and g odd
    // swap:   (f, g) <- (g, (g - f)/2);  odd: g <- (g + f)/2;  even: g <- g/2
    g += ((f ^ c) - c) & godd;
    q += ((u ^ c) - c) & godd;
    r += ((v ^ c) - c) & godd;
    f += g & c;
    u += q & c;
    v += r & c;
    delta = (int32_t)(((uint32_t)delta ^ c) - c) + 1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  u_ = (int32_t)u; v_ = (int32_t)v; q_ = (int32_t)q; r_ = (int32_t)r;
}

BGV_HD void s30_update_fg(s30_t& f, s30_t& g, int32_t u, int32_t v, int32_t q, int32_t r) {
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;  // exact: the low 30 bits are zero by construction
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 13; i++) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)(cf & S30_MASK);
    g.v[i - 1] = (int32_t)(cg & S30_MASK);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[12] = (int32_t)cf;
  g.v[12] = (int32_t)cg;
}

// (d, e) <- ([u v; q r] (d, e) + (md, me) p) / 2^30 with md, me making the
// low limb vanish; d, e stay in (-2p, p): first add p for each negative input
// (|u d~ + v e~| < 2^30 p), then subtract t p with t in [0, 2^30).
BGV_HD void s30_update_de(s30_t& d, s30_t& e, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t sd = d.v[12] >> 31, se = e.v[12] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((P_INV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)S30_MASK);
  me -= (int32_t)((P_INV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)S30_MASK);
  cd += (int64_t)P_S30[0] * md;
  ce += (int64_t)P_S30[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 13; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)P_S30[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)P_S30[i] * me;
    d.v[i - 1] = (int32_t)(cd & S30_MASK);
    e.v[i - 1] = (int32_t)(ce & S30_MASK);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[12] = (int32_t)cd;
  e.v[12] = (int32_t)ce;
}

// d <- d + (p & mask) (mask 0 or -1), limbs renormalized
BGV_HD void s30_add_p_masked(s30_t& d, int32_t mask) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    c += (int64_t)d.v[i] + (P_S30[i] & mask);
    d.v[i] = (int32_t)(c & S30_MASK);
    c >>= 30;
  }
  d.v[12] = (int32_t)(c + d.v[12] + (P_S30[12] & mask));
}

BGV_HD bool s30_is_zero(const s30_t& a) {
  int32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 13; i++) acc |= a.v[i];
  return acc == 0;
}

// r = a^-1 in the Montgomery domain (0 -> 0).  The divsteps invert the plain
// integer aR; (aR)^-1 R^3 / R = a^-1 R.
BGV_NI void fp_inv(fp_t& r, const fp_t& a) {
  s30_t f, g, d, e;
#pragma unroll
  for (int i = 0; i < 13; i++) {
    f.v[i] = P_S30[i];
    d.v[i] = 0;
    e.v[i] = 0;
  }
  e.v[0] = 1;
  s30_from_fp(g, a);
  int32_t delta = 1;
  for (int it = 0; it < 37; it++) {
    int32_t u, v, q, rr;
    divsteps30(delta, (uint32_t)f.v[0], (uint32_t)g.v[0], u, v, q, rr);
    s30_update_de(d, e, u, v, q, rr);
    s30_update_fg(f, g, u, v, q, rr);
    if (s30_is_zero(g)) break;
  }
  // f = +-1: negate d when f < 0, then bring (-2p, 2p) into [0, p)
  const int32_t neg = f.v[12] >> 31;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    c += (int64_t)((d.v[i] ^ neg) - neg);
    d.v[i] = (int32_t)(c & S30_MASK);
    c >>= 30;
  }
  d.v[12] = (int32_t)(c + ((d.v[12] ^ neg) - neg));
  s30_add_p_masked(d, d.v[12] >> 31);
  s30_add_p_masked(d, d.v[12] >> 31);
  s30_t t = d;
  {
    int64_t b = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      b += (int64_t)t.v[i] - P_S30[i];
      t.v[i] = (int32_t)(b & S30_MASK);
      b >>= 30;
    }
    t.v[12] = (int32_t)(b + t.v[12] - P_S30[12]);
  }
  if (t.v[12] >= 0) d = t;  // d >= p
  fp_t x;
  s30_to_fp(x, d);
  fp_mul(r, x, R3_MOD);
}

// ---- digit form for exponentiation chains -----------------------------------
// A chain of products needs no additions, so between its products an element
// can stay in the product's own 14 x 28-bit digit form: no unpack / pack and
// no final subtraction per product (fd leaf 498 instructions against 618;
// tools/ubench_fd.hip: 13% lower lone-wave latency, 12% more products/s).
// fd_t holds v 2^392 mod p (Montgomery with R = 2^392, no pre-shift) as 14
// signed digits; every value here is a product output: digits 0..12 in
// [0, 2^28), digit 13 the small non-negative rest, value < 1.001 p (inputs
// < 1.1 p: the Montgomery sum is < 1.1^2 p^2 / 2^392 + p).
struct fd_t { int32_t d[14]; };
BGV_CONST uint32_t FD_K400[14] = {0x80e6299u, 0x3500034u, 0xeb12856u, 0xdeb2699u, 0xc988670u, 0x4ef6697u, 0x70983e8u,
                                  0xa4e6fe9u, 0x3e8a053u, 0xecf271eu, 0xc20d323u, 0x6eb6385u, 0x47f1286u, 0x156dau};  // 2^400 mod p
BGV_CONST uint32_t FD_K384[14] = {0x2fffdu, 0x900000u, 0xc000276u, 0xbc40u, 0x8baebf4u, 0x5753c75u, 0x55f4898u,
                                  0x7052574u, 0x7ce5853u, 0x56ec6d7u, 0x71a97a2u, 0xe4935c0u, 0xec3fa80u, 0x15f65u};  // 2^384 mod p

// r = a b / 2^392: signed product scanning, Montgomery reduction by 2^28 per digit
template <class V>
BGV_HD void fd_mul_core(V& r, const V& a, const V& b) {
  uint64_t acc[28];
#pragma unroll
  for (int k = 0; k < 28; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++)
#pragma unroll
    for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)((int64_t)a[i] * (int64_t)b[j]);
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t m = ((uint32_t)acc[i] * P28_INV) & M28;
#pragma unroll
    for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += (uint64_t)((int64_t)acc[i] >> 28);
  }
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int64_t v = (int64_t)acc[14 + k] + c;
    r[k] = (int32_t)(v & M28);
    c = v >> 28;
  }
  r[13] = (int32_t)((int64_t)acc[27] + c);
}

// squaring: the 91 cross products once against a doubled digit
template <class V>
BGV_HD void fd_sqr_core(V& r, const V& a) {
  uint64_t acc[28];
#pragma unroll
  for (int k = 0; k < 28; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    acc[2 * i] += (uint64_t)((int64_t)a[i] * (int64_t)a[i]);
#pragma unroll
    for (int j = i + 1; j < 14; j++) acc[i + j] += (uint64_t)((int64_t)a[i] * (int64_t)(2 * a[j]));
  }
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const uint32_t m = ((uint32_t)acc[i] * P28_INV) & M28;
#pragma unroll
    for (int j = 0; j < 14; j++) acc[i + j] += (uint64_t)m * P28[j];
    acc[i + 1] += (uint64_t)((int64_t)acc[i] >> 28);
  }
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int64_t v = (int64_t)acc[14 + k] + c;
    r[k] = (int32_t)(v & M28);
    c = v >> 28;
  }
  r[13] = (int32_t)((int64_t)acc[27] + c);
}

#if defined(__HIPCC__) && BGV_FPMUL_CALL
// register-ABI leaves like fp_mul_leaf (operands v0-v27, result v0-v13)
typedef int32_t fd_vec_t __attribute__((ext_vector_type(14)));
static __device__ __noinline__ fd_vec_t fd_mul_leaf(fd_vec_t a, fd_vec_t b) {
  fd_vec_t r;
  fd_mul_core(r, a, b);
  return r;
}
static __device__ __noinline__ fd_vec_t fd_sqr_leaf(fd_vec_t a) {
  fd_vec_t r;
  fd_sqr_core(r, a);
  return r;
}
#endif

BGV_HD void fd_mul(fd_t& r, const fd_t& a, const fd_t& b) {
#ifdef BGV_COUNT_OPS
  bgv_fpmul_count++;
#endif
#if defined(__HIP_DEVICE_COMPILE__) && BGV_FPMUL_CALL
  fd_vec_t va, vb;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    va[k] = a.d[k];
    vb[k] = b.d[k];
  }
  const fd_vec_t vr = fd_mul_leaf(va, vb);
#pragma unroll
  for (int k = 0; k < 14; k++) r.d[k] = vr[k];
#else
  fd_t t;
  fd_mul_core(t.d, a.d, b.d);
  r = t;
#endif
}

BGV_HD void fd_sqr(fd_t& r, const fd_t& a) {
#ifdef BGV_COUNT_OPS
  bgv_fpmul_count++;
#endif
#if defined(__HIP_DEVICE_COMPILE__) && BGV_FPMUL_CALL
  fd_vec_t va;
#pragma unroll
  for (int k = 0; k < 14; k++) va[k] = a.d[k];
  const fd_vec_t vr = fd_sqr_leaf(va);
#pragma unroll
  for (int k = 0; k < 14; k++) r.d[k] = vr[k];
#else
  fd_t t;
  fd_sqr_core(t.d, a.d);
  r = t;
#endif
}

// a R (R = 2^384, canonical) -> a 2^392 in digit form: its digits times 2^400
BGV_HD void fd_from_fp(fd_t& r, const fp_t& a) {
  uint32_t u[14];
  unpack28<0>(u, a);
  fd_t x, k;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    x.d[i] = (int32_t)u[i];
    k.d[i] = (int32_t)FD_K400[i];
  }
  fd_mul(r, x, k);
}

// v 2^392 -> v R canonical (one product by 2^384, then one conditional
// subtraction of p: the product is < 1.001 p)
BGV_HD void fd_to_fp(fp_t& r, const fd_t& a) {
  fd_t k, t;
#pragma unroll
  for (int i = 0; i < 14; i++) k.d[i] = (int32_t)FD_K384[i];
  fd_mul(t, a, k);
  uint32_t d[14], u[14];
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int32_t v = t.d[i] - (int32_t)P28[i] - borrow;
    borrow = v < 0 && i < 13 ? 1 : 0;
    u[i] = (uint32_t)(i < 13 ? (v & (int32_t)M28) : v);
    d[i] = (uint32_t)t.d[i];
  }
  const bool ge = (int32_t)u[13] >= 0;  // t >= p
#pragma unroll
  for (int i = 0; i < 14; i++) d[i] = ge ? u[i] : d[i];
  pack28(r, d);
}

// r = a^e for a fixed exponent given as a 4-bit sliding-window plan
// (tools/gen_constants.py pow_plan): odd powers a, a^3, ..., a^15, then per
// step `shift` squarings and one product by a table entry.  The plan is the
// same for every lane, so the table entry is chosen by a scalar branch and
// the table stays in registers.  (p+1)/4: 378 squarings + 86 products
// (+8 for the table) against 378 + 228 for plain binary.  The chain runs in
// the digit form (2 extra products for the conversions).
#ifndef BGV_FD_POW
#define BGV_FD_POW 1
#endif
#if BGV_FD_POW
#define POW_T fd_t
#define POW_MUL fd_mul
#define POW_SQR fd_sqr
#else
#define POW_T fp_t
#define POW_MUL fp_mul
#define POW_SQR fp_sqr
#endif
BGV_NI void fp_pow_plan(fp_t& r, const fp_t& a_in, const uint8_t* shift, const uint8_t* idx, uint32_t n, uint32_t first) {
  POW_T t[8], a2;
#if BGV_FD_POW
  fd_from_fp(t[0], a_in);
#else
  t[0] = a_in;
#endif
  POW_SQR(a2, t[0]);
#pragma unroll
  for (int k = 1; k < 8; k++) POW_MUL(t[k], t[k - 1], a2);
  POW_T acc = t[0];
#pragma unroll
  for (int k = 1; k < 8; k++)
    if (first == (uint32_t)k) acc = t[k];
  for (uint32_t s = 0; s < n; s++) {
    const uint32_t sh = shift[s];
    for (uint32_t k = 0; k < sh; k++) POW_SQR(acc, acc);
    switch (idx[s]) {
      case 0: POW_MUL(acc, acc, t[0]); break;
      case 1: POW_MUL(acc, acc, t[1]); break;
      case 2: POW_MUL(acc, acc, t[2]); break;
      case 3: POW_MUL(acc, acc, t[3]); break;
      case 4: POW_MUL(acc, acc, t[4]); break;
      case 5: POW_MUL(acc, acc, t[5]); break;
      case 6: POW_MUL(acc, acc, t[6]); break;
      case 7: POW_MUL(acc, acc, t[7]); break;
      default: break;
    }
  }
#if BGV_FD_POW
  fd_to_fp(r, acc);
#else
  r = acc;
#endif
}
#undef POW_T
#undef POW_MUL
#undef POW_SQR

// a^((p+1)/4) and a^((p-3)/4)
BGV_HD void fp_pow_sqrt(fp_t& r, const fp_t& a) { fp_pow_plan(r, a, POWP_SQRT_SHIFT, POWP_SQRT_IDX, POWP_SQRT_N, POWP_SQRT_FIRST); }
BGV_HD void fp_pow_sqrt_tail(fp_t& r, const fp_t& a) {
  fp_pow_plan(r, a, POWP_SQRT_TAIL_SHIFT, POWP_SQRT_TAIL_IDX, POWP_SQRT_TAIL_N, POWP_SQRT_TAIL_FIRST);
}

// candidate square root a^((p+1)/4); returns true iff it squares back to a
BGV_HD bool fp_sqrt(fp_t& r, const fp_t& a) {
  fp_t s, chk;
  fp_pow_sqrt(s, a);
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
  for (int i = 0; i < NL; i++) (void)subb32(a.l[i], P_MOD.l[i], borrow, borrow);
  return borrow != 0;
}

// plain-integer comparison a > (p-1)/2 (ZCash "lexicographically largest")
BGV_HD bool fp_plain_gt_half(const fp_t& a) {
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) (void)subb32(P_HALF.l[i], a.l[i], borrow, borrow);
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
