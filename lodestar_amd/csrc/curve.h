// G1 (over Fp) and G2 (over Fp2) short-Weierstrass y^2 = x^3 + b in Jacobian
// coordinates.  One templated set of formulas serves both groups.
//
// Reference operations re-created here (all inside third-party blst, reached
// from the reference at these call sites):
//   * bls.PublicKey.aggregate           chain/bls/utils.ts:11
//   * Signature.fromBytes(.., validate) chain/bls/maybeBatch.ts:23,36
//     (G2 decompression + subgroup check)
//   * mul_n_aggregate 64-bit scalars    chain/bls/maybeBatch.ts:18
#pragma once
#include "fp12.h"

// point additions/doublings: inlined into the bulk kernels (BGV_POINT_INLINE,
// bgv_kernels.hip) so their Fp2 temporaries stay in registers around the
// register-ABI product leaf; non-inlined elsewhere
#if defined(__HIPCC__) && BGV_POINT_INLINE
#define BGV_NIP BGV_HD
#else
#define BGV_NIP BGV_NI
#endif
// scalar-multiplication-level routines (x-chains, subgroup / cofactor maps,
// affine conversion): BGV_CURVE_INLINE inlines them too (A/B knob)
#if defined(__HIPCC__) && BGV_CURVE_INLINE
#define BGV_NIC BGV_HD
#else
#define BGV_NIC BGV_NI
#endif

namespace bgv {

// ---- field overloads used by the generic point code ------------------------
BGV_HD void fe_add(fp_t& r, const fp_t& a, const fp_t& b) { fp_add(r, a, b); }
BGV_HD void fe_sub(fp_t& r, const fp_t& a, const fp_t& b) { fp_sub(r, a, b); }
BGV_HD void fe_dbl(fp_t& r, const fp_t& a) { fp_dbl(r, a); }
BGV_HD void fe_mul(fp_t& r, const fp_t& a, const fp_t& b) { fp_mul(r, a, b); }
BGV_HD void fe_sqr(fp_t& r, const fp_t& a) { fp_sqr(r, a); }
BGV_HD void fe_neg(fp_t& r, const fp_t& a) { fp_neg(r, a); }
BGV_HD void fe_inv(fp_t& r, const fp_t& a) { fp_inv(r, a); }
BGV_HD bool fe_is_zero(const fp_t& a) { return fp_is_zero(a); }
BGV_HD bool fe_eq(const fp_t& a, const fp_t& b) { return fp_eq(a, b); }
BGV_HD void fe_zero(fp_t& r) { fp_set_zero(r); }
BGV_HD void fe_one(fp_t& r) { r = FP_ONE; }
BGV_HD void fe_select(fp_t& r, bool c, const fp_t& a, const fp_t& b) { fp_select(r, c, a, b); }

BGV_HD void fe_add(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp2_add(r, a, b); }
BGV_HD void fe_sub(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp2_sub(r, a, b); }
BGV_HD void fe_dbl(fp2_t& r, const fp2_t& a) { fp2_dbl(r, a); }
BGV_HD void fe_mul(fp2_t& r, const fp2_t& a, const fp2_t& b) { fp2_mul(r, a, b); }
BGV_HD void fe_sqr(fp2_t& r, const fp2_t& a) { fp2_sqr(r, a); }
BGV_HD void fe_neg(fp2_t& r, const fp2_t& a) { fp2_neg(r, a); }
BGV_HD void fe_inv(fp2_t& r, const fp2_t& a) { fp2_inv(r, a); }
BGV_HD bool fe_is_zero(const fp2_t& a) { return fp2_is_zero(a); }
BGV_HD bool fe_eq(const fp2_t& a, const fp2_t& b) { return fp2_eq(a, b); }
BGV_HD void fe_zero(fp2_t& r) { r = fp2_zero(); }
BGV_HD void fe_one(fp2_t& r) { r = fp2_one(); }
BGV_HD void fe_select(fp2_t& r, bool c, const fp2_t& a, const fp2_t& b) { fp2_select(r, c, a, b); }

template <class F> struct jac_t { F x, y, z; };
template <class F> struct aff_t { F x, y; };

template <class F> BGV_HD bool jac_is_inf(const jac_t<F>& p) { return fe_is_zero(p.z); }

template <class F> BGV_HD void jac_set_inf(jac_t<F>& p) {
  fe_one(p.x); fe_one(p.y); fe_zero(p.z);
}

template <class F> BGV_HD void jac_from_aff(jac_t<F>& r, const aff_t<F>& a) {
  r.x = a.x; r.y = a.y; fe_one(r.z);
}

template <class F> BGV_HD void jac_neg(jac_t<F>& r, const jac_t<F>& p) {
  r.x = p.x; fe_neg(r.y, p.y); r.z = p.z;
}

// dbl-2009-l (a = 0): 2M + 5S
template <class F> BGV_NIP void jac_dbl(jac_t<F>& r, const jac_t<F>& p) {
  F A, B, C, D, E, Fq, t;
  fe_sqr(A, p.x);
  fe_sqr(B, p.y);
  fe_sqr(C, B);
  fe_add(t, p.x, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_dbl(D, t);
  fe_dbl(E, A);
  fe_add(E, E, A);
  fe_sqr(Fq, E);
  F x3, y3, z3;
  fe_dbl(t, D);
  fe_sub(x3, Fq, t);
  fe_sub(t, D, x3);
  fe_mul(y3, E, t);
  fe_dbl(C, C); fe_dbl(C, C); fe_dbl(C, C);
  fe_sub(y3, y3, C);
  fe_mul(z3, p.y, p.z);
  fe_dbl(z3, z3);
  r.x = x3; r.y = y3; r.z = z3;
}

// add-2007-bl with the exceptional cases (infinity, P == Q, P == -Q)
template <class F> BGV_NIP void jac_add(jac_t<F>& r, const jac_t<F>& p, const jac_t<F>& q) {
  if (jac_is_inf(p)) { r = q; return; }
  if (jac_is_inf(q)) { r = p; return; }
  F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fe_sqr(z1z1, p.z);
  fe_sqr(z2z2, q.z);
  fe_mul(u1, p.x, z2z2);
  fe_mul(u2, q.x, z1z1);
  fe_mul(s1, p.y, q.z);
  fe_mul(s1, s1, z2z2);
  fe_mul(s2, q.y, p.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, u1);
  fe_sub(rr, s2, s1);
  if (fe_is_zero(h)) {
    if (fe_is_zero(rr)) { jac_dbl(r, p); return; }
    jac_set_inf(r);
    return;
  }
  fe_dbl(i, h);
  fe_sqr(i, i);
  fe_mul(j, h, i);
  fe_dbl(rr, rr);
  fe_mul(v, u1, i);
  F x3, y3, z3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, s1, j);
  fe_dbl(t, t);
  fe_sub(y3, y3, t);
  fe_add(z3, p.z, q.z);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, z2z2);
  fe_mul(z3, z3, h);
  r.x = x3; r.y = y3; r.z = z3;
}

// madd-2007-bl: Jacobian + affine (q not infinity), with exceptional cases
template <class F> BGV_NIP void jac_add_aff(jac_t<F>& r, const jac_t<F>& p, const aff_t<F>& q) {
  if (jac_is_inf(p)) { jac_from_aff(r, q); return; }
  F z1z1, u2, s2, h, hh, i, j, rr, v, t;
  fe_sqr(z1z1, p.z);
  fe_mul(u2, q.x, z1z1);
  fe_mul(s2, q.y, p.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, p.x);
  fe_sub(rr, s2, p.y);
  if (fe_is_zero(h)) {
    if (fe_is_zero(rr)) { jac_dbl(r, p); return; }
    jac_set_inf(r);
    return;
  }
  fe_sqr(hh, h);
  fe_dbl(i, hh);
  fe_dbl(i, i);
  fe_mul(j, h, i);
  fe_dbl(rr, rr);
  fe_mul(v, p.x, i);
  F x3, y3, z3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, p.y, j);
  fe_dbl(t, t);
  fe_sub(y3, y3, t);
  fe_add(z3, p.z, h);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, hh);
  r.x = x3; r.y = y3; r.z = z3;
}

// [k]P for a public/random 64-bit scalar k (left-to-right double-and-add)
template <class F> BGV_NI void jac_mul_u64(jac_t<F>& r, const jac_t<F>& p, uint64_t k) {
  jac_t<F> acc;
  jac_set_inf(acc);
  if (k == 0) { r = acc; return; }
  int top = 63;
  while (!((k >> top) & 1ull)) top--;
  acc = p;
  for (int b = top - 1; b >= 0; b--) {
    jac_dbl(acc, acc);
    if ((k >> b) & 1ull) jac_add(acc, acc, p);
  }
  r = acc;
}

// [k]P for a RANDOM 64-bit scalar (the batch multipliers r_i), fixed 4-bit
// window with a per-lane table {O, P, .., 15P}.  Double-and-add branches on
// each lane's own bits, so a wave executes the addition at almost every bit
// (64 dbl + ~64 add); here every lane runs the same 60 dbl + 15 add + 14
// table steps.
template <class F> BGV_NI void jac_mul_u64_w4(jac_t<F>& r, const jac_t<F>& p, uint64_t k) {
  jac_t<F> tab[16];
  jac_set_inf(tab[0]);
  tab[1] = p;
  jac_dbl(tab[2], p);
#pragma unroll 1
  for (int i = 3; i < 16; i++) jac_add(tab[i], tab[i - 1], p);
  jac_t<F> acc = tab[(k >> 60) & 15];
#pragma unroll 1
  for (int w = 14; w >= 0; w--) {
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    jac_dbl(acc, acc);
    const jac_t<F> t = tab[(k >> (4 * w)) & 15];
    jac_add(acc, acc, t);
  }
  r = acc;
}

// the addition in the x-chain and the cofactor map.  As a call (one copy per
// unit, BGV_ADD_CALL_INLINE=0) its temporaries do not share a frame with the
// doubling's, but every call saves and restores the callee-saved VGPRs
// through scratch; inlined, k_hash's frame grows (5,168 -> 6,224 B) and C4
// still runs 0.25 ms faster (profiles/r05f_add_call_inline_ab.txt: 37.57
// against 37.32 ms, A/B over three alternating pairs on one box)
#ifndef BGV_ADD_CALL_INLINE
#define BGV_ADD_CALL_INLINE 1
#endif
#if defined(__HIPCC__) && BGV_ADD_CALL_INLINE
template <class F> BGV_HD void jac_add_call(jac_t<F>& r, const jac_t<F>& p, const jac_t<F>& q) { jac_add(r, p, q); }
#else
template <class F> BGV_NI void jac_add_call(jac_t<F>& r, const jac_t<F>& p, const jac_t<F>& q) { jac_add(r, p, q); }
#endif

// [|x|]P for the BLS parameter: |x| = 0xd201000000010000 has its bits 63,
// 62, 60, 57, 48 and 16 set, so after the top bit the double-and-add is runs
// of 1, 2, 3, 9, 32 doublings, each followed by an addition, then 16
// doublings (the same operations as the bitwise loop, in the same order)
template <class F> BGV_NIC void jac_mul_abs_x(jac_t<F>& r, const jac_t<F>& p) {
  static_assert(BLS_X_ABS_C == 0xd201000000010000ull, "x-chain runs");
  jac_t<F> acc = p;
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int run = s == 0 ? 1 : (s == 1 ? 2 : (s == 2 ? 3 : (s == 3 ? 9 : (s == 4 ? 32 : 16))));
#pragma unroll 1
    for (int k = 0; k < run; k++) jac_dbl(acc, acc);
    if (s < 5) jac_add_call(acc, acc, p);
  }
  r = acc;
}

template <class F> BGV_NIC bool jac_to_aff(aff_t<F>& r, const jac_t<F>& p) {
  if (jac_is_inf(p)) { fe_zero(r.x); fe_zero(r.y); return false; }
  F zi, zi2, zi3;
  fe_inv(zi, p.z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(r.x, p.x, zi2);
  fe_mul(r.y, p.y, zi3);
  return true;
}

// equality of two Jacobian points (cross-multiplied)
template <class F> BGV_NIC bool jac_eq(const jac_t<F>& p, const jac_t<F>& q) {
  const bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F z1z1, z2z2, a, b;
  fe_sqr(z1z1, p.z);
  fe_sqr(z2z2, q.z);
  fe_mul(a, p.x, z2z2);
  fe_mul(b, q.x, z1z1);
  if (!fe_eq(a, b)) return false;
  fe_mul(a, p.y, q.z);
  fe_mul(a, a, z2z2);
  fe_mul(b, q.y, p.z);
  fe_mul(b, b, z1z1);
  return fe_eq(a, b);
}

using g1j = jac_t<fp_t>;
using g1a = aff_t<fp_t>;
using g2j = jac_t<fp2_t>;
using g2a = aff_t<fp2_t>;

// ---- G2 endomorphism psi and the subgroup check ---------------------------

BGV_HD void g2_psi(g2j& r, const g2j& p) {
  // psi works coordinate-wise on Jacobian points too: x/z^2 -> conj(x)/conj(z)^2 * cx
  fp2_t x, y, z;
  fp2_conj(x, p.x);
  fp2_conj(y, p.y);
  fp2_conj(z, p.z);
  fp2_mul(r.x, x, PSI_CX);
  fp2_mul(r.y, y, PSI_CY);
  r.z = z;
}

BGV_HD void g2_psi2(g2j& r, const g2j& p) {
  fp2_mul_fp(r.x, p.x, PSI2_CX);
  fp2_mul_fp(r.y, p.y, PSI2_CY);
  r.z = p.z;
}

// Scott's test: P in G2  <=>  psi(P) == [x]P  (x = -|x|)
BGV_NIC bool g2_in_subgroup(const g2j& p) {
  if (jac_is_inf(p)) return true;
  g2j xp, ps;
  jac_mul_abs_x(xp, p);
  jac_neg(xp, xp);
  g2_psi(ps, p);
  return jac_eq(ps, xp);
}

BGV_HD bool g2_aff_on_curve(const g2a& a) {
  fp2_t l, rr;
  fp2_sqr(l, a.y);
  fp2_sqr(rr, a.x);
  fp2_mul(rr, rr, a.x);
  fp2_add(rr, rr, B2_MONT);
  return fp2_eq(l, rr);
}

// h_eff [P] = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)  (Budroni-Pintore)
BGV_NIC void g2_clear_cofactor(g2j& r, const g2j& p) {
  g2j t1, t2, t3, np;
  jac_mul_abs_x(t1, p);
  jac_neg(t1, t1);            // [x]P
  jac_mul_abs_x(t2, t1);
  jac_neg(t2, t2);            // [x^2]P
  jac_neg(np, p);
  jac_add_call(t3, t1, np);        // [x - 1]P
  g2_psi(t3, t3);             // psi([x-1]P)
  jac_neg(t1, t1);
  jac_add_call(t2, t2, t1);        // [x^2 - x]P
  jac_add_call(t2, t2, np);        // [x^2 - x - 1]P
  jac_add_call(t2, t2, t3);
  jac_dbl(t1, p);
  g2_psi2(t1, t1);
  jac_add_call(r, t2, t1);
}

// ---- serialization ---------------------------------------------------------
// blst error codes (bindings/blst.h BLST_ERROR) + @chainsafe/blst size error
enum : int32_t {
  C_OK = 0,
  C_BAD_ENCODING = 1,
  C_POINT_NOT_ON_CURVE = 2,
  C_POINT_NOT_IN_GROUP = 3,
  C_AGGR_TYPE_MISMATCH = 4,
  C_VERIFY_FAIL = 5,
  C_PK_IS_INFINITY = 6,
  C_BAD_SCALAR = 7,
  C_INVALID_SIZE = 8,
};

// ZCash 96-byte compressed G2 -> affine (Montgomery) ; returns BGV_* code.
// *inf set for the canonical infinity encoding.
BGV_NI int32_t g2_decompress(g2a& out, bool& inf, const uint8_t* b) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return C_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 96; i++) acc |= b[i];
    if (acc) return C_BAD_ENCODING;
    inf = true;
    out.x = fp2_zero(); out.y = fp2_zero();
    return C_OK;
  }
  fp_t x1, x0;
  fp_from_be48(x1, b);
  x1.l[NL - 1] &= 0x1fffffffu;  // clear the 3 flag bits
  fp_from_be48(x0, b + 48);
  if (!fp_plain_lt_p(x1) || !fp_plain_lt_p(x0)) return C_BAD_ENCODING;
  fp2_t x, y2, y;
  fp_to_mont(x.c0, x0);
  fp_to_mont(x.c1, x1);
  fp2_sqr(y2, x);
  fp2_mul(y2, y2, x);
  fp2_add(y2, y2, B2_MONT);
  if (!fp2_sqrt(y, y2)) return C_POINT_NOT_ON_CURVE;
  const bool want_large = (b0 & 0x20) != 0;
  if (fp2_lex_largest(y) != want_large) fp2_neg(y, y);
  out.x = x;
  out.y = y;
  return C_OK;
}

// 192-byte uncompressed G2 (blst POINTonE2_Deserialize_Z behind
// @chainsafe/blst's Signature.fromBytes: a 192-byte input must not carry the
// compression flag (P2_Affine rejects len != (in[0] & 0x80 ? 96 : 192)), the
// infinity flag needs every other bit zero, and any other flag bit is
// BAD_ENCODING)
BGV_NI int32_t g2_deserialize(g2a& out, bool& inf, const uint8_t* b) {
  inf = false;
  const uint8_t b0 = b[0];
  if (b0 & 0x80) return C_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 192; i++) acc |= b[i];
    if (acc) return C_BAD_ENCODING;
    inf = true;
    out.x = fp2_zero(); out.y = fp2_zero();
    return C_OK;
  }
  if (b0 & 0x20) return C_BAD_ENCODING;  // a sign bit only exists on compressed encodings
  fp_t x1, x0, y1, y0;
  fp_from_be48(x1, b);
  x1.l[NL - 1] &= 0x1fffffffu;
  fp_from_be48(x0, b + 48);
  fp_from_be48(y1, b + 96);
  fp_from_be48(y0, b + 144);
  if (!fp_plain_lt_p(x1) || !fp_plain_lt_p(x0) || !fp_plain_lt_p(y1) || !fp_plain_lt_p(y0)) return C_BAD_ENCODING;
  fp_to_mont(out.x.c0, x0);
  fp_to_mont(out.x.c1, x1);
  fp_to_mont(out.y.c0, y0);
  fp_to_mont(out.y.c1, y1);
  if (!g2_aff_on_curve(out)) return C_POINT_NOT_ON_CURVE;
  return C_OK;
}

// 96-byte uncompressed G1 (x || y big-endian, the pool's PointFormat.uncompressed,
// multithread/index.ts:132,177), trusted: no curve/subgroup validation, like
// PublicKey.fromBytes(.., affine) in multithread/worker.ts:108-114.
BGV_HD bool g1_from_uncompressed_trusted(g1a& out, const uint8_t* b) {
  if (b[0] & 0x40) return false;  // infinity
  fp_t x, y;
  fp_from_be48(x, b);
  x.l[NL - 1] &= 0x1fffffffu;
  fp_from_be48(y, b + 48);
  fp_to_mont(out.x, x);
  fp_to_mont(out.y, y);
  return true;
}

// 48-byte compressed G1 (trusted table entry: decompress, no subgroup check)
BGV_NI int32_t g1_decompress(g1a& out, bool& inf, const uint8_t* b) {
  inf = false;
  const uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return C_BAD_ENCODING;
  if (b0 & 0x40) {
    uint32_t acc = b0 & 0x3f;
    for (int i = 1; i < 48; i++) acc |= b[i];
    if (acc) return C_BAD_ENCODING;
    inf = true;
    fp_set_zero(out.x); fp_set_zero(out.y);
    return C_OK;
  }
  fp_t x;
  fp_from_be48(x, b);
  x.l[NL - 1] &= 0x1fffffffu;
  if (!fp_plain_lt_p(x)) return C_BAD_ENCODING;
  fp_t xm, y2, y;
  fp_to_mont(xm, x);
  fp_sqr(y2, xm);
  fp_mul(y2, y2, xm);
  fp_add(y2, y2, B1_MONT);
  if (!fp_sqrt(y, y2)) return C_POINT_NOT_ON_CURVE;
  if (fp_lex_largest(y) != ((b0 & 0x20) != 0)) fp_neg(y, y);
  out.x = xm;
  out.y = y;
  return C_OK;
}

}  // namespace bgv
