// hash_to_G2 for the Ethereum BLS ciphersuite
//   DST = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"
// RFC 9380 suite BLS12381G2_XMD:SHA-256_SSWU_RO_: expand_message_xmd with
// SHA-256 (on-device compression function), hash_to_field (2 x Fp2),
// simplified SWU onto E2', the 3-isogeny to E2 and clear_cofactor (h_eff via
// the psi endomorphism).  Re-creates the hashing blst performs inside
// Pairing::mul_n_aggregate / aggregate (packages/beacon-node/src/chain/bls/
// maybeBatch.ts:18,37).  Signing roots are always 32 bytes
// (ISignatureSet.signingRoot: Root, state-transition/src/util/signatureSets.ts:13).
#pragma once
#include "curve.h"

#if defined(__HIPCC__) && BGV_H2C_INLINE
#define BGV_NIH BGV_HD
#else
#define BGV_NIH BGV_NI
#endif

namespace bgv {

BGV_CONST uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

BGV_CONST uint32_t SHA256_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// DST_prime = DST || len(DST) = 44 bytes
BGV_CONST uint8_t DST_PRIME[44] = {'B', 'L', 'S', '_', 'S', 'I', 'G', '_', 'B', 'L', 'S', '1', '2', '3', '8',
                                   '1', 'G', '2', '_', 'X', 'M', 'D', ':', 'S', 'H', 'A', '-', '2', '5', '6',
                                   '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 'P', 'O', 'P', '_', 43};

BGV_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// one SHA-256 compression of a 16-word big-endian block
BGV_NI void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + SHA256_K[i] + wi;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// write byte v at big-endian byte position pos of a 16-word block
BGV_HD void blk_put(uint32_t blk[16], int pos, uint32_t v) {
  blk[pos >> 2] |= (v & 0xffu) << (24 - 8 * (pos & 3));
}

BGV_HD void blk_clear(uint32_t blk[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) blk[i] = 0;
}

// expand_message_xmd(msg[32], DST, 256) -> 64 big-endian words
BGV_NI void expand_message_xmd_256(uint32_t out[64], const uint8_t msg[32]) {
  uint32_t blk[16];
  uint32_t st[8];
  // b0 = H(Z_pad[64] || msg[32] || I2OSP(256, 2) || 0x00 || DST_prime[44]): 143 bytes, 3 blocks
#pragma unroll
  for (int i = 0; i < 8; i++) st[i] = SHA256_IV[i];
  blk_clear(blk);
  sha256_compress(st, blk);  // the all-zero Z_pad block
  blk_clear(blk);
  for (int i = 0; i < 32; i++) blk_put(blk, i, msg[i]);
  blk_put(blk, 32, 0x01);
  blk_put(blk, 33, 0x00);
  blk_put(blk, 34, 0x00);
  for (int i = 0; i < 29; i++) blk_put(blk, 35 + i, DST_PRIME[i]);
  sha256_compress(st, blk);
  blk_clear(blk);
  for (int i = 0; i < 15; i++) blk_put(blk, i, DST_PRIME[29 + i]);
  blk_put(blk, 15, 0x80);
  blk[15] = 143u * 8u;
  sha256_compress(st, blk);
  uint32_t b0[8];
#pragma unroll
  for (int i = 0; i < 8; i++) b0[i] = st[i];
  // b_i = H((b0 ^ b_{i-1}) || I2OSP(i, 1) || DST_prime): 77 bytes, 2 blocks
  uint32_t prev[8];
#pragma unroll
  for (int i = 0; i < 8; i++) prev[i] = 0;  // b0 ^ 0 = b0 for i = 1
  for (int i = 1; i <= 8; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) st[k] = SHA256_IV[k];
    blk_clear(blk);
#pragma unroll
    for (int k = 0; k < 8; k++) blk[k] = b0[k] ^ prev[k];
    blk_put(blk, 32, (uint32_t)i);
    for (int k = 0; k < 31; k++) blk_put(blk, 33 + k, DST_PRIME[k]);
    sha256_compress(st, blk);
    blk_clear(blk);
    for (int k = 0; k < 13; k++) blk_put(blk, k, DST_PRIME[31 + k]);
    blk_put(blk, 13, 0x80);
    blk[15] = 77u * 8u;
    sha256_compress(st, blk);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      prev[k] = st[k];
      out[(i - 1) * 8 + k] = st[k];
    }
  }
}

// 16 big-endian words (64 bytes) -> Fp (Montgomery), e mod p
BGV_HD void fp_from_be512_words(fp_t& r, const uint32_t w[16]) {
  fp_t hi, lo, a, b;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    hi.l[i] = w[7 - i];
    lo.l[i] = w[15 - i];
  }
#pragma unroll
  for (int i = 8; i < NL; i++) { hi.l[i] = 0; lo.l[i] = 0; }
  fp_mul(a, hi, H2F_K);
  fp_mul(b, lo, R2_MOD);
  fp_add(r, a, b);
}

BGV_HD void hash_to_field_fp2x2(fp2_t& u0, fp2_t& u1, const uint8_t msg[32]) {
  uint32_t ub[64];
  expand_message_xmd_256(ub, msg);
  fp_from_be512_words(u0.c0, ub + 0);
  fp_from_be512_words(u0.c1, ub + 16);
  fp_from_be512_words(u1.c0, ub + 32);
  fp_from_be512_words(u1.c1, ub + 48);
}

// simplified SWU onto E2' (RFC 9380 6.6.2), affine output
BGV_NIH void map_to_curve_sswu(g2a& out, const fp2_t& u) {
  fp2_t u2, zu2, den, tv1, x1, x2, gx1, gx2, t;
  fp2_sqr(u2, u);
  fp2_mul(zu2, SSWU_Z, u2);
  fp2_sqr(den, zu2);
  fp2_add(den, den, zu2);
  if (fp2_is_zero(den)) {
    x1 = SSWU_B_OVER_ZA;
  } else {
    fp2_inv(tv1, den);
    fp2_add(tv1, tv1, fp2_one());
    fp2_mul(x1, SSWU_MINUS_B_OVER_A, tv1);
  }
  // gx1 = x1^3 + A x1 + B
  fp2_sqr(t, x1);
  fp2_add(t, t, SSWU_A);
  fp2_mul(gx1, t, x1);
  fp2_add(gx1, gx1, SSWU_B);
  fp2_mul(x2, zu2, x1);
  fp2_sqr(t, x2);
  fp2_add(t, t, SSWU_A);
  fp2_mul(gx2, t, x2);
  fp2_add(gx2, gx2, SSWU_B);
  // gx1 is a square in Fp2 iff norm(gx1) is one in Fp, and the root of the
  // norm is the first half of fp2_sqrt anyway: one exponentiation answers the
  // test and starts the root.  Otherwise d^2 = -norm(gx1) and, as
  // gx2 = Z^3 u^6 gx1, sqrt(norm(gx2)) = sqrt(-norm(Z)^3) norm(u)^3 d.
  // (RFC 9380 6.6.2 computes is_square(gx1) and sqrt() separately: 4 exponentiations.)
  fp_t n1, d, chk, nu, nu3, d2;
  fp2_norm(n1, gx1);
  fp_pow_sqrt(d, n1);
  fp_sqr(chk, d);
  const bool sq = fp_eq(chk, n1);
  fp2_norm(nu, u);
  fp_sqr(nu3, nu);
  fp_mul(nu3, nu3, nu);
  fp_mul(d2, d, nu3);
  fp_mul(d2, d2, SSWU_SQRT_NEG_NZ3);
  fp2_t x, g, y;
  fp2_select(x, sq, x1, x2);
  fp2_select(g, sq, gx1, gx2);
  if (!sq) d = d2;
  // exceptional u (den == 0: x1 = B/(ZA), the gx2 identity does not hold) and
  // g with a zero imaginary part take the general root
  if (fp_is_zero(g.c1) || (!sq && fp2_is_zero(den))) fp2_sqrt(y, g);
  else fp2_sqrt_tail(y, g, d);
  if (fp2_sgn0(u) != fp2_sgn0(y)) fp2_neg(y, y);
  out.x = x;
  out.y = y;
}

template <int N>
BGV_HD void fp2_horner(fp2_t& r, const fp2_t (&c)[N], const fp2_t& x) {
  fp2_t acc = c[N - 1];
#pragma unroll
  for (int i = N - 2; i >= 0; i--) {
    fp2_mul(acc, acc, x);
    fp2_add(acc, acc, c[i]);
  }
  r = acc;
}

// 3-isogeny E2' -> E2 straight into Jacobian coordinates (no inversion):
// Z = xden yden, X = xnum xden yden^2, Y = y ynum xden^3 yden^2
BGV_NIH void iso_map_g2(g2j& r, const g2a& p) {
  fp2_t xn, xd, yn, yd, t, yd2;
  fp2_horner(xn, ISO_XNUM, p.x);
  fp2_horner(xd, ISO_XDEN, p.x);
  fp2_horner(yn, ISO_YNUM, p.x);
  fp2_horner(yd, ISO_YDEN, p.x);
  fp2_mul(r.z, xd, yd);
  fp2_sqr(yd2, yd);
  fp2_mul(t, xn, xd);
  fp2_mul(r.x, t, yd2);
  fp2_sqr(t, xd);
  fp2_mul(t, t, xd);
  fp2_mul(t, t, yd2);
  fp2_mul(t, t, yn);
  fp2_mul(r.y, t, p.y);
}

// split form for small batches (two lanes per message): lane k in {0, 1}
// maps u_k through SSWU and the isogeny; hash_to_g2_finish adds the two
// points and clears the cofactor.  Same values as hash_to_g2.
BGV_NI void hash_to_g2_map(g2j& out, const uint8_t msg[32], uint32_t k) {
  fp2_t u0, u1;
  hash_to_field_fp2x2(u0, u1, msg);
  g2a qa;
  map_to_curve_sswu(qa, k ? u1 : u0);
  iso_map_g2(out, qa);
}

BGV_NI void hash_to_g2_finish(g2j& out, const g2j& q0, const g2j& q1) {
  g2j r;
  jac_add(r, q0, q1);
  g2_clear_cofactor(out, r);
}

// full hash_to_G2(msg[32]) -> Jacobian point in G2
BGV_NI void hash_to_g2(g2j& out, const uint8_t msg[32]) {
  fp2_t u0, u1;
  hash_to_field_fp2x2(u0, u1, msg);
  g2a q0a, q1a;
  map_to_curve_sswu(q0a, u0);
  map_to_curve_sswu(q1a, u1);
  g2j q0, q1, r;
  iso_map_g2(q0, q0a);
  iso_map_g2(q1, q1a);
  jac_add(r, q0, q1);
  g2_clear_cofactor(out, r);
}

}  // namespace bgv
