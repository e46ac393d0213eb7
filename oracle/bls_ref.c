/*
 * bls_ref.c -- CPU restatement of the BLS12-381 batch signature-set
 * verification the reference reaches through @chainsafe/bls 7.1.1 ->
 * @chainsafe/blst 0.2.8 -> supranational blst (un-vendored; call sites
 * packages/beacon-node/src/chain/bls/maybeBatch.ts:16-38,
 * chain/bls/utils.ts:5-16).
 *
 * TEST INFRASTRUCTURE ONLY (oracle/).  Used by tests/ as a checker at sizes
 * the Python oracle cannot reach, and by bench.py's cpu_baseline leg as the
 * host-core baseline ("port": same algorithms, 6 x 64-bit limbs with
 * 128-bit products, -O3 -march=native, one job per thread like the
 * reference's worker pool, multithread/worker.ts:30-106).  Never linked into
 * the product.  Pinned against oracle/bls12_381.py (itself pinned to the
 * reference's KATs) by tests/test_cref.py.
 *
 * Semantics restated:
 *   Signature.fromBytes(sig, affine, validate=true): 96 B compressed /
 *     192 B uncompressed ZCash encodings, BLST_BAD_ENCODING /
 *     POINT_NOT_ON_CURVE / POINT_NOT_IN_GROUP / INVALID_SIZE
 *   verifyMultipleSignatures: e(-G1, sum r_i sig_i) * prod e(r_i pk_i, H(m_i)) == 1
 *   verify (1 set): e(-G1, sig) * e(pk, H(m)) == 1
 *   hash_to_G2: RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_ with the POP DST
 */
#include <stdint.h>
#include <x86intrin.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>
#include "bls_ref_consts.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t l[6]; } fp;
typedef struct { fp c0, c1; } fp2;
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
typedef struct { fp x, y, z; } g1j;
typedef struct { fp x, y; int inf; } g1a;
typedef struct { fp2 x, y, z; } g2j;
typedef struct { fp2 x, y; int inf; } g2a;

static const uint64_t PM[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                               0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
static const uint64_t PINV = 0x89f3fffcfffcfffdull; /* -p^-1 mod 2^64 */
static const uint64_t RORD[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                 0x73eda753299d7d48ull};
static const uint64_t XABS = 0xd201000000010000ull;

static fp R1, R2, FONE, FHALF, T256;
static fp E_PM2, E_SQRT, E_LEG, E_P34;
static fp2 B2M, B2X3, G2X, G2Y, PSI_X, PSI_Y, PSI2_X, PSI2_Y, FROB[3][5], S_A, S_B, S_Z, S_MBA, S_BZA;
static fp2 IXN[4], IXD[3], IYN[4], IYD[4];
static g1a G1A, G1NEG;
static int inited = 0;

/* ------------------------------------------------------------------ Fp */
static int fp_is_zero(const fp* a) { return !(a->l[0] | a->l[1] | a->l[2] | a->l[3] | a->l[4] | a->l[5]); }
static int fp_eq(const fp* a, const fp* b) { return !memcmp(a, b, sizeof(fp)); }
static int geq_p(const uint64_t* a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > PM[i]) return 1;
    if (a[i] < PM[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t* a) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - PM[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}
/* modular add / sub on adc / sbb chains, branch-free selection */
static inline void fp_add(fp* r, const fp* a, const fp* b) {
  unsigned long long t[6], u[6];
  unsigned char c = 0, br = 0;
  for (int i = 0; i < 6; i++) c = _addcarry_u64(c, a->l[i], b->l[i], &t[i]);
  for (int i = 0; i < 6; i++) br = _subborrow_u64(br, t[i], PM[i], &u[i]);
  const uint64_t keep = -(uint64_t)br; /* t < p: keep t (a + b < 2p < 2^384: no carry out) */
  for (int i = 0; i < 6; i++) r->l[i] = (t[i] & keep) | (u[i] & ~keep);
}
static inline void fp_sub(fp* r, const fp* a, const fp* b) {
  unsigned long long t[6];
  unsigned char br = 0, c = 0;
  for (int i = 0; i < 6; i++) br = _subborrow_u64(br, a->l[i], b->l[i], &t[i]);
  const uint64_t m = -(uint64_t)br;
  for (int i = 0; i < 6; i++) c = _addcarry_u64(c, t[i], PM[i] & m, (unsigned long long*)&r->l[i]);
}
static inline void fp_neg(fp* r, const fp* a) {
  static const fp z;
  fp_sub(r, &z, a);
}
#include "bls_ref_mulx.h"
static uint64_t PMX[7]; /* p, then -p^-1 mod 2^64 (fp_mul_mulx) */
static int use_mulx = 0; /* the CPU has BMI2 + ADX (bref_init) */
static void fp_mul_portable(fp* r, const fp* a, const fp* b);
static inline void fp_mul(fp* r, const fp* a, const fp* b) {
  if (use_mulx) fp_mul_mulx(r->l, a->l, b->l, PMX);
  else fp_mul_portable(r, a, b);
}
static void fp_mul_portable(fp* r, const fp* a, const fp* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 6; j++) {
      u128 s = (u128)a->l[j] * b->l[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[6] + c;
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * PINV;
    s = (u128)m * PM[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < 6; j++) {
      s = (u128)m * PM[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[6] + c;
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  if (t[6] || geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}
static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
/* a^e, 4-bit fixed window (e plain, 6 limbs) */
static void fp_pow(fp* r, const fp* a, const fp* e) {
  fp tab[16], acc = FONE;
  tab[0] = FONE;
  tab[1] = *a;
  for (int i = 2; i < 16; i++) fp_mul(&tab[i], &tab[i - 1], a);
  int started = 0;
  for (int w = 95; w >= 0; w--) {
    const unsigned d = (unsigned)(e->l[w >> 4] >> (4 * (w & 15))) & 15u;
    if (started) {
      fp_sqr(&acc, &acc); fp_sqr(&acc, &acc); fp_sqr(&acc, &acc); fp_sqr(&acc, &acc);
      if (d) fp_mul(&acc, &acc, &tab[d]);
    } else if (d) {
      acc = tab[d];
      started = 1;
    }
  }
  *r = acc;
}
/* plain 6-limb helpers for the binary inversion */
static inline int u384_is_one(const uint64_t* a) { return a[0] == 1 && !(a[1] | a[2] | a[3] | a[4] | a[5]); }
static inline int u384_geq(const uint64_t* a, const uint64_t* b) {
  for (int i = 5; i >= 0; i--) if (a[i] != b[i]) return a[i] > b[i];
  return 1;
}
static inline void u384_sub(uint64_t* a, const uint64_t* b) {
  unsigned char br = 0;
  for (int i = 0; i < 6; i++) br = _subborrow_u64(br, a[i], b[i], (unsigned long long*)&a[i]);
}
static inline void u384_shr1(uint64_t* a) {
  for (int i = 0; i < 5; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 63);
  a[5] >>= 1;
}
/* x / 2 mod p for x < p (plain) */
static inline void half_mod_p(uint64_t* x) {
  if (x[0] & 1) {
    unsigned char c = 0;
    unsigned long long t[6];
    for (int i = 0; i < 6; i++) c = _addcarry_u64(c, x[i], PM[i], &t[i]);
    for (int i = 0; i < 5; i++) x[i] = (t[i] >> 1) | (t[i + 1] << 63);
    x[5] = (t[5] >> 1) | ((uint64_t)c << 63);
  } else {
    u384_shr1(x);
  }
}
static fp R3; /* R^3 mod p, Montgomery form of R^2 */
/* Montgomery inverse by the binary extended Euclid on the plain value A = aR:
 * x = A^-1 mod p, then x R^3 R^-1 = R^2 / A = a^-1 R.  Not constant time: the
 * oracle and the CPU baseline verify public data. */
static void fp_inv(fp* r, const fp* a) {
  uint64_t u[6], v[6], x1[6] = {1, 0, 0, 0, 0, 0}, x2[6] = {0};
  memcpy(u, a->l, 48);
  memcpy(v, PM, 48);
  if (!(u[0] | u[1] | u[2] | u[3] | u[4] | u[5])) { memset(r, 0, sizeof *r); return; }
  while (!u384_is_one(u) && !u384_is_one(v)) {
    while (!(u[0] & 1)) { u384_shr1(u); half_mod_p(x1); }
    while (!(v[0] & 1)) { u384_shr1(v); half_mod_p(x2); }
    if (u384_geq(u, v)) {
      u384_sub(u, v);
      fp_sub((fp*)x1, (const fp*)x1, (const fp*)x2);
    } else {
      u384_sub(v, u);
      fp_sub((fp*)x2, (const fp*)x2, (const fp*)x1);
    }
  }
  fp x;
  memcpy(x.l, u384_is_one(u) ? x1 : x2, 48);
  fp_mul(r, &x, &R3);
}
static int fp_sqrt(fp* r, const fp* a) {
  fp s, c;
  fp_pow(&s, a, &E_SQRT);
  fp_sqr(&c, &s);
  *r = s;
  return fp_eq(&c, a);
}
static void fp_from_be(fp* r, const uint8_t* b) {
  for (int i = 0; i < 6; i++) {
    uint64_t w = 0;
    for (int k = 0; k < 8; k++) w = (w << 8) | b[40 - 8 * i + k];
    r->l[i] = w;
  }
}
static void fp_to_be(uint8_t* b, const fp* a) {
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[40 - 8 * i + k] = (uint8_t)(a->l[i] >> (56 - 8 * k));
}
static void to_mont(fp* r, const fp* a) { fp_mul(r, a, &R2); }
static void from_mont(fp* r, const fp* a) {
  fp one;
  memset(&one, 0, sizeof one);
  one.l[0] = 1;
  fp_mul(r, a, &one);
}
static int lex_gt_half(const fp* m) { /* plain value > (p-1)/2 */
  fp t;
  from_mont(&t, m);
  fp h = E_LEG; /* (p-1)/2 */
  for (int i = 5; i >= 0; i--) {
    if (t.l[i] > h.l[i]) return 1;
    if (t.l[i] < h.l[i]) return 0;
  }
  return 0;
}
static int fp_parity(const fp* m) {
  fp t;
  from_mont(&t, m);
  return (int)(t.l[0] & 1);
}
static void hex_to_fp(fp* r, const char* h) { /* 96 hex chars, big-endian, -> Montgomery */
  uint8_t b[48];
  for (int i = 0; i < 48; i++) {
    int v = 0;
    for (int k = 0; k < 2; k++) {
      char c = h[2 * i + k];
      v = v * 16 + (c <= '9' ? c - '0' : (c | 32) - 'a' + 10);
    }
    b[i] = (uint8_t)v;
  }
  fp t;
  fp_from_be(&t, b);
  to_mont(r, &t);
}

/* ----------------------------------------------------------------- Fp2 */
static void f2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void f2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void f2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void f2_dbl(fp2* r, const fp2* a) { f2_add(r, a, a); }
static void f2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static int f2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int f2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void f2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, t2, t3;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&t2, &a->c0, &a->c1);
  fp_add(&t3, &b->c0, &b->c1);
  fp_mul(&t2, &t2, &t3);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&t2, &t2, &t0);
  fp_sub(&r->c1, &t2, &t1);
}
static void f2_sqr(fp2* r, const fp2* a) {
  fp t0, t1, t2;
  fp_add(&t0, &a->c0, &a->c1);
  fp_sub(&t1, &a->c0, &a->c1);
  fp_mul(&t2, &a->c0, &a->c1);
  fp_mul(&r->c0, &t0, &t1);
  fp_add(&r->c1, &t2, &t2);
}
static void f2_mul_fp(fp2* r, const fp2* a, const fp* b) { fp_mul(&r->c0, &a->c0, b); fp_mul(&r->c1, &a->c1, b); }
static void f2_mul_xi(fp2* r, const fp2* a) {
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static void f2_norm(fp* r, const fp2* a) {
  fp t0, t1;
  fp_sqr(&t0, &a->c0);
  fp_sqr(&t1, &a->c1);
  fp_add(r, &t0, &t1);
}
static void f2_inv(fp2* r, const fp2* a) {
  fp n, t;
  f2_norm(&n, a);
  fp_inv(&n, &n);
  fp_mul(&r->c0, &a->c0, &n);
  fp_mul(&t, &a->c1, &n);
  fp_neg(&r->c1, &t);
}
/* Fp2 square root by two Fp exponentiations (p = 3 mod 4), the norm method
 * of the device (lodestar_amd/csrc/fp2.h fp2_sqrt): d = sqrt(a0^2 + a1^2)
 * exists iff a is a square; t = (a0 + d)/2, s = t^((p-3)/4); s^2 t == 1 gives
 * x = s t + (a1 s / 2) i, otherwise x = (a1 s / 2) - (s t) i.  Any root is
 * fine: callers fix the sign (sgn0 / lexicographic flag). */
static void f2_sqrt_tail(fp2* r, const fp2* a, const fp* d) {
  fp t, s, st, s2t, as;
  fp_add(&t, &a->c0, d);
  fp_mul(&t, &t, &FHALF);
  fp_pow(&s, &t, &E_P34);
  fp_mul(&st, &s, &t);
  fp_mul(&s2t, &st, &s);
  fp_mul(&as, &a->c1, &s);
  fp_mul(&as, &as, &FHALF);
  if (fp_eq(&s2t, &FONE)) { r->c0 = st; r->c1 = as; }
  else { r->c0 = as; fp_neg(&r->c1, &st); }
}
static int f2_sqrt(fp2* r, const fp2* a) {
  if (fp_is_zero(&a->c1)) {
    fp s;
    if (fp_sqrt(&s, &a->c0)) { r->c0 = s; memset(&r->c1, 0, sizeof(fp)); return 1; }
    fp na;
    fp_neg(&na, &a->c0); /* -1 is a non-residue: -a0 is a square, x = sqrt(-a0) i */
    fp_sqrt(&s, &na);
    memset(&r->c0, 0, sizeof(fp));
    r->c1 = s;
    return 1;
  }
  fp n, d;
  f2_norm(&n, a);
  if (!fp_sqrt(&d, &n)) return 0;
  f2_sqrt_tail(r, a, &d);
  return 1;
}
static int f2_sgn0(const fp2* a) {
  int s0 = fp_parity(&a->c0), z0 = fp_is_zero(&a->c0), s1 = fp_parity(&a->c1);
  return s0 | (z0 & s1);
}
static int f2_lex(const fp2* a) { return fp_is_zero(&a->c1) ? lex_gt_half(&a->c0) : lex_gt_half(&a->c1); }

/* ------------------------------------------------------------ Fp6, Fp12 */
static void f6_add(fp6* r, const fp6* a, const fp6* b) { f2_add(&r->c0, &a->c0, &b->c0); f2_add(&r->c1, &a->c1, &b->c1); f2_add(&r->c2, &a->c2, &b->c2); }
static void f6_sub(fp6* r, const fp6* a, const fp6* b) { f2_sub(&r->c0, &a->c0, &b->c0); f2_sub(&r->c1, &a->c1, &b->c1); f2_sub(&r->c2, &a->c2, &b->c2); }
static void f6_neg(fp6* r, const fp6* a) { f2_neg(&r->c0, &a->c0); f2_neg(&r->c1, &a->c1); f2_neg(&r->c2, &a->c2); }
static void f6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  f2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void f6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 t0, t1, t2, s0, s1, u, c0, c1, c2;
  f2_mul(&t0, &a->c0, &b->c0);
  f2_mul(&t1, &a->c1, &b->c1);
  f2_mul(&t2, &a->c2, &b->c2);
  f2_add(&s0, &a->c1, &a->c2); f2_add(&s1, &b->c1, &b->c2); f2_mul(&u, &s0, &s1);
  f2_sub(&u, &u, &t1); f2_sub(&u, &u, &t2); f2_mul_xi(&u, &u); f2_add(&c0, &u, &t0);
  f2_add(&s0, &a->c0, &a->c1); f2_add(&s1, &b->c0, &b->c1); f2_mul(&u, &s0, &s1);
  f2_sub(&u, &u, &t0); f2_sub(&u, &u, &t1); f2_mul_xi(&s0, &t2); f2_add(&c1, &u, &s0);
  f2_add(&s0, &a->c0, &a->c2); f2_add(&s1, &b->c0, &b->c2); f2_mul(&u, &s0, &s1);
  f2_sub(&u, &u, &t0); f2_sub(&u, &u, &t2); f2_add(&c2, &u, &t1);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
static void f6_inv(fp6* r, const fp6* a) {
  fp2 c0, c1, c2, t, n;
  f2_sqr(&c0, &a->c0); f2_mul(&t, &a->c1, &a->c2); f2_mul_xi(&t, &t); f2_sub(&c0, &c0, &t);
  f2_sqr(&c1, &a->c2); f2_mul_xi(&c1, &c1); f2_mul(&t, &a->c0, &a->c1); f2_sub(&c1, &c1, &t);
  f2_sqr(&c2, &a->c1); f2_mul(&t, &a->c0, &a->c2); f2_sub(&c2, &c2, &t);
  f2_mul(&n, &a->c2, &c1); f2_mul(&t, &a->c1, &c2); f2_add(&n, &n, &t); f2_mul_xi(&n, &n);
  f2_mul(&t, &a->c0, &c0); f2_add(&n, &n, &t); f2_inv(&n, &n);
  f2_mul(&r->c0, &c0, &n); f2_mul(&r->c1, &c1, &n); f2_mul(&r->c2, &c2, &n);
}
static void f12_one(fp12* r) {
  memset(r, 0, sizeof *r);
  r->c0.c0.c0 = FONE;
}
static int f12_is_one(const fp12* a) {
  fp12 o;
  f12_one(&o);
  return !memcmp(a, &o, sizeof o);
}
static void f12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s0, s1;
  f6_mul(&t0, &a->c0, &b->c0);
  f6_mul(&t1, &a->c1, &b->c1);
  f6_add(&s0, &a->c0, &a->c1);
  f6_add(&s1, &b->c0, &b->c1);
  f6_mul(&s0, &s0, &s1);
  f6_sub(&s0, &s0, &t0);
  f6_sub(&r->c1, &s0, &t1);
  f6_mul_v(&t1, &t1);
  f6_add(&r->c0, &t0, &t1);
}
static void f12_sqr(fp12* r, const fp12* a) {
  fp6 t0, t1, t2;
  f6_mul(&t0, &a->c0, &a->c1);
  f6_add(&t1, &a->c0, &a->c1);
  f6_mul_v(&t2, &a->c1);
  f6_add(&t2, &a->c0, &t2);
  f6_mul(&t1, &t1, &t2);
  f6_sub(&t1, &t1, &t0);
  f6_mul_v(&t2, &t0);
  f6_sub(&r->c0, &t1, &t2);
  f6_add(&r->c1, &t0, &t0);
}
static void f12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; f6_neg(&r->c1, &a->c1); }
static void f12_inv(fp12* r, const fp12* a) {
  fp6 t0, t1;
  f6_mul(&t0, &a->c0, &a->c0);
  f6_mul(&t1, &a->c1, &a->c1);
  f6_mul_v(&t1, &t1);
  f6_sub(&t0, &t0, &t1);
  f6_inv(&t0, &t0);
  f6_mul(&r->c0, &a->c0, &t0);
  f6_mul(&t1, &a->c1, &t0);
  f6_neg(&r->c1, &t1);
}
/* multiply by the sparse line l = a0 + a1 w^2 + b1 w^3, i.e. l0 = (a0, a1, 0)
 * and l1 = (0, b1, 0) in Fp12 = Fp6[w]: Karatsuba over w with sparse Fp6
 * products, 13 Fp2 multiplications instead of 18 */
static void f6_mul_01(fp6* r, const fp6* a, const fp2* b0, const fp2* b1) { /* a * (b0 + b1 v) */
  fp2 t0, t1, u, s0, s1, c0, c1, c2;
  f2_mul(&t0, &a->c0, b0);
  f2_mul(&t1, &a->c1, b1);
  f2_add(&s0, &a->c1, &a->c2); f2_mul(&u, &s0, b1); f2_sub(&u, &u, &t1); f2_mul_xi(&u, &u); f2_add(&c0, &u, &t0);
  f2_add(&s0, &a->c0, &a->c1); f2_add(&s1, b0, b1); f2_mul(&u, &s0, &s1); f2_sub(&u, &u, &t0); f2_sub(&c1, &u, &t1);
  f2_add(&s0, &a->c0, &a->c2); f2_mul(&u, &s0, b0); f2_sub(&u, &u, &t0); f2_add(&c2, &u, &t1);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
static void f6_mul_1(fp6* r, const fp6* a, const fp2* b1) { /* a * (b1 v) */
  fp2 c0, c1, c2;
  f2_mul(&c0, &a->c2, b1); f2_mul_xi(&c0, &c0);
  f2_mul(&c1, &a->c0, b1);
  f2_mul(&c2, &a->c1, b1);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
static void f12_mul_line(fp12* f, const fp2* a0, const fp2* a1, const fp2* b1) {
  fp6 t0, t1, s;
  fp2 ab;
  f6_mul_01(&t0, &f->c0, a0, a1);
  f6_mul_1(&t1, &f->c1, b1);
  f6_add(&s, &f->c0, &f->c1);
  f2_add(&ab, a1, b1);
  f6_mul_01(&s, &s, a0, &ab);
  f6_sub(&s, &s, &t0);
  f6_sub(&f->c1, &s, &t1);
  f6_mul_v(&t1, &t1);
  f6_add(&f->c0, &t0, &t1);
}
static void f12_frob(fp12* r, const fp12* a, int k) {
  fp2 c[6] = {a->c0.c0, a->c1.c0, a->c0.c1, a->c1.c1, a->c0.c2, a->c1.c2};
  for (int i = 0; i < 6; i++) {
    if (k & 1) f2_conj(&c[i], &c[i]);
    if (i) f2_mul(&c[i], &c[i], &FROB[k - 1][i - 1]);
  }
  r->c0.c0 = c[0]; r->c1.c0 = c[1]; r->c0.c1 = c[2]; r->c1.c1 = c[3]; r->c0.c2 = c[4]; r->c1.c2 = c[5];
}
static void f4_sqr(fp2* r0, fp2* r1, const fp2* a, const fp2* b) {
  fp2 t0, t1, t2;
  f2_sqr(&t0, a); f2_sqr(&t1, b); f2_mul_xi(&t2, &t1); f2_add(r0, &t2, &t0);
  f2_add(&t2, a, b); f2_sqr(&t2, &t2); f2_sub(&t2, &t2, &t0); f2_sub(r1, &t2, &t1);
}
static void f12_cyc_sqr(fp12* r, const fp12* f) {
  fp2 z0 = f->c0.c0, z1 = f->c1.c1, z2 = f->c1.c0, z3 = f->c0.c2, z4 = f->c0.c1, z5 = f->c1.c2;
  fp2 t0, t1, t2, t3, u;
  f4_sqr(&t0, &t1, &z0, &z1);
  f2_sub(&u, &t0, &z0); f2_dbl(&u, &u); f2_add(&z0, &u, &t0);
  f2_add(&u, &t1, &z1); f2_dbl(&u, &u); f2_add(&z1, &u, &t1);
  f4_sqr(&t0, &t1, &z2, &z3);
  f4_sqr(&t2, &t3, &z4, &z5);
  f2_sub(&u, &t0, &z4); f2_dbl(&u, &u); f2_add(&z4, &u, &t0);
  f2_add(&u, &t1, &z5); f2_dbl(&u, &u); f2_add(&z5, &u, &t1);
  f2_mul_xi(&t0, &t3);
  f2_add(&u, &t0, &z2); f2_dbl(&u, &u); f2_add(&z2, &u, &t0);
  f2_sub(&u, &t2, &z3); f2_dbl(&u, &u); f2_add(&z3, &u, &t2);
  r->c0.c0 = z0; r->c1.c1 = z1; r->c1.c0 = z2; r->c0.c2 = z3; r->c0.c1 = z4; r->c1.c2 = z5;
}
static void f12_pow_x(fp12* r, const fp12* a) {
  fp12 acc = *a;
  for (int b = 62; b >= 0; b--) {
    f12_cyc_sqr(&acc, &acc);
    if ((XABS >> b) & 1) f12_mul(&acc, &acc, a);
  }
  f12_conj(r, &acc);
}
static void final_exp(fp12* r, const fp12* f) {
  fp12 t0, t1, y0, y1, y2, y3;
  f12_inv(&t0, f); f12_conj(&t1, f); f12_mul(&t1, &t1, &t0);
  f12_frob(&t0, &t1, 2); f12_mul(&t1, &t0, &t1);
  f12_pow_x(&t0, &t1); f12_conj(&y0, &t1); f12_mul(&y0, &t0, &y0);
  f12_pow_x(&t0, &y0); f12_conj(&y1, &y0); f12_mul(&y1, &t0, &y1);
  f12_pow_x(&t0, &y1); f12_frob(&y2, &y1, 1); f12_mul(&y2, &t0, &y2);
  f12_pow_x(&t0, &y2); f12_pow_x(&t0, &t0); f12_frob(&y3, &y2, 2); f12_mul(&y3, &t0, &y3);
  f12_conj(&t0, &y2); f12_mul(&y3, &y3, &t0);
  f12_cyc_sqr(&t0, &t1); f12_mul(&t0, &t0, &t1); f12_mul(r, &y3, &t0);
}

/* ---------------------------------------------------------- curves */
#define JAC_IMPL(G, F, ADD, SUB, MUL, SQR, DBLF, ISZ, EQ, ONE_SET, ONE_Z)                         \
  static void G##_dbl(G* r, const G* p) {                                                  \
    F A, B, C, D, E, FF, t, x3, y3, z3;                                                    \
    SQR(&A, &p->x); SQR(&B, &p->y); SQR(&C, &B);                                           \
    ADD(&t, &p->x, &B); SQR(&t, &t); SUB(&t, &t, &A); SUB(&t, &t, &C); DBLF(&D, &t);       \
    DBLF(&E, &A); ADD(&E, &E, &A); SQR(&FF, &E);                                           \
    DBLF(&t, &D); SUB(&x3, &FF, &t); SUB(&t, &D, &x3); MUL(&y3, &E, &t);                   \
    DBLF(&C, &C); DBLF(&C, &C); DBLF(&C, &C); SUB(&y3, &y3, &C);                           \
    MUL(&z3, &p->y, &p->z); DBLF(&z3, &z3);                                                \
    r->x = x3; r->y = y3; r->z = z3;                                                       \
  }                                                                                        \
  static void G##_add(G* r, const G* p, const G* q) {                                      \
    if (ISZ(&p->z)) { *r = *q; return; }                                                   \
    if (ISZ(&q->z)) { *r = *p; return; }                                                   \
    F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t, x3, y3, z3;                           \
    SQR(&z1z1, &p->z); SQR(&z2z2, &q->z); MUL(&u1, &p->x, &z2z2); MUL(&u2, &q->x, &z1z1);  \
    MUL(&s1, &p->y, &q->z); MUL(&s1, &s1, &z2z2); MUL(&s2, &q->y, &p->z); MUL(&s2, &s2, &z1z1); \
    SUB(&h, &u2, &u1); SUB(&rr, &s2, &s1);                                                 \
    if (ISZ(&h)) {                                                                         \
      if (ISZ(&rr)) { G##_dbl(r, p); return; }                                             \
      ONE_SET(r); return;                                                                  \
    }                                                                                      \
    DBLF(&i, &h); SQR(&i, &i); MUL(&j, &h, &i); DBLF(&rr, &rr); MUL(&v, &u1, &i);           \
    SQR(&x3, &rr); SUB(&x3, &x3, &j); SUB(&x3, &x3, &v); SUB(&x3, &x3, &v);                \
    SUB(&t, &v, &x3); MUL(&y3, &rr, &t); MUL(&t, &s1, &j); DBLF(&t, &t); SUB(&y3, &y3, &t); \
    ADD(&z3, &p->z, &q->z); SQR(&z3, &z3); SUB(&z3, &z3, &z1z1); SUB(&z3, &z3, &z2z2);     \
    MUL(&z3, &z3, &h);                                                                     \
    r->x = x3; r->y = y3; r->z = z3;                                                       \
  }                                                                                        \
  /* p + (qx, qy, 1) (madd-2007-bl); same exceptional cases */                             \
  static void G##_add_aff(G* r, const G* p, const F* qx, const F* qy) {                    \
    if (ISZ(&p->z)) { r->x = *qx; r->y = *qy; ONE_Z(&r->z); return; }                      \
    F z1z1, u2, s2, h, hh, i, j, rr, v, t, x3, y3, z3;                                     \
    SQR(&z1z1, &p->z); MUL(&u2, qx, &z1z1); MUL(&s2, qy, &p->z); MUL(&s2, &s2, &z1z1);     \
    SUB(&h, &u2, &p->x); SUB(&rr, &s2, &p->y);                                             \
    if (ISZ(&h)) {                                                                         \
      if (ISZ(&rr)) { G##_dbl(r, p); return; }                                             \
      ONE_SET(r); return;                                                                  \
    }                                                                                      \
    SQR(&hh, &h); DBLF(&i, &hh); DBLF(&i, &i); MUL(&j, &h, &i); DBLF(&rr, &rr);             \
    MUL(&v, &p->x, &i);                                                                    \
    SQR(&x3, &rr); SUB(&x3, &x3, &j); SUB(&x3, &x3, &v); SUB(&x3, &x3, &v);                \
    SUB(&t, &v, &x3); MUL(&y3, &rr, &t); MUL(&t, &p->y, &j); DBLF(&t, &t); SUB(&y3, &y3, &t); \
    ADD(&z3, &p->z, &h); SQR(&z3, &z3); SUB(&z3, &z3, &z1z1); SUB(&z3, &z3, &hh);          \
    r->x = x3; r->y = y3; r->z = z3;                                                       \
  }

static void fp_dbl(fp* r, const fp* a) { fp_add(r, a, a); }
static void g1_set_inf(g1j* r) { r->x = FONE; r->y = FONE; memset(&r->z, 0, sizeof(fp)); }
static void g2_set_inf(g2j* r) {
  memset(r, 0, sizeof *r);
  r->x.c0 = FONE;
  r->y.c0 = FONE;
}
static void fp_one_z(fp* z) { *z = FONE; }
static void f2_one_z(fp2* z) { memset(z, 0, sizeof *z); z->c0 = FONE; }
JAC_IMPL(g1j, fp, fp_add, fp_sub, fp_mul, fp_sqr, fp_dbl, fp_is_zero, fp_eq, g1_set_inf, fp_one_z)
JAC_IMPL(g2j, fp2, f2_add, f2_sub, f2_mul, f2_sqr, f2_dbl, f2_is_zero, f2_eq, g2_set_inf, f2_one_z)

static void g1_from_aff(g1j* r, const g1a* a) { r->x = a->x; r->y = a->y; r->z = FONE; }
static void g2_from_aff(g2j* r, const g2a* a) {
  r->x = a->x; r->y = a->y;
  memset(&r->z, 0, sizeof(fp2));
  r->z.c0 = FONE;
}
static void g1_to_aff(g1a* r, const g1j* p) {
  if (fp_is_zero(&p->z)) { memset(r, 0, sizeof *r); r->inf = 1; return; }
  fp zi, z2, z3;
  fp_inv(&zi, &p->z); fp_sqr(&z2, &zi); fp_mul(&z3, &z2, &zi);
  fp_mul(&r->x, &p->x, &z2); fp_mul(&r->y, &p->y, &z3); r->inf = 0;
}
static void g2_to_aff(g2a* r, const g2j* p) {
  if (f2_is_zero(&p->z)) { memset(r, 0, sizeof *r); r->inf = 1; return; }
  fp2 zi, z2, z3;
  f2_inv(&zi, &p->z); f2_sqr(&z2, &zi); f2_mul(&z3, &z2, &zi);
  f2_mul(&r->x, &p->x, &z2); f2_mul(&r->y, &p->y, &z3); r->inf = 0;
}
/* [k]P by double-and-add; mixed additions when P has Z = 1 */
static void g1_mul_u64(g1j* r, const g1j* p, uint64_t k) {
  g1j acc;
  g1_set_inf(&acc);
  const int aff = fp_eq(&p->z, &FONE);
  for (int b = 63; b >= 0; b--) {
    g1j_dbl(&acc, &acc);
    if ((k >> b) & 1) {
      if (aff) g1j_add_aff(&acc, &acc, &p->x, &p->y);
      else g1j_add(&acc, &acc, p);
    }
  }
  *r = acc;
}
static void g2_mul_u64(g2j* r, const g2j* p, uint64_t k) {
  g2j acc;
  g2_set_inf(&acc);
  fp2 one;
  f2_one_z(&one);
  const int aff = f2_eq(&p->z, &one);
  for (int b = 63; b >= 0; b--) {
    g2j_dbl(&acc, &acc);
    if ((k >> b) & 1) {
      if (aff) g2j_add_aff(&acc, &acc, &p->x, &p->y);
      else g2j_add(&acc, &acc, p);
    }
  }
  *r = acc;
}
static void g2_mul_words(g2j* r, const g2j* p, const uint64_t* k, int nw) {
  g2j acc;
  g2_set_inf(&acc);
  for (int w = nw - 1; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      g2j_dbl(&acc, &acc);
      if ((k[w] >> b) & 1) g2j_add(&acc, &acc, p);
    }
  *r = acc;
}
static void g1_mul_words(g1j* r, const g1j* p, const uint64_t* k, int nw) {
  g1j acc;
  g1_set_inf(&acc);
  for (int w = nw - 1; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      g1j_dbl(&acc, &acc);
      if ((k[w] >> b) & 1) g1j_add(&acc, &acc, p);
    }
  *r = acc;
}
static int g2_eq(const g2j* p, const g2j* q) {
  int pi = f2_is_zero(&p->z), qi = f2_is_zero(&q->z);
  if (pi || qi) return pi && qi;
  fp2 a, b, z1, z2;
  f2_sqr(&z1, &p->z); f2_sqr(&z2, &q->z);
  f2_mul(&a, &p->x, &z2); f2_mul(&b, &q->x, &z1);
  if (!f2_eq(&a, &b)) return 0;
  f2_mul(&a, &p->y, &q->z); f2_mul(&a, &a, &z2); f2_mul(&b, &q->y, &p->z); f2_mul(&b, &b, &z1);
  return f2_eq(&a, &b);
}
static void g2_psi(g2j* r, const g2j* p) {
  fp2 x, y, z;
  f2_conj(&x, &p->x); f2_conj(&y, &p->y); f2_conj(&z, &p->z);
  f2_mul(&r->x, &x, &PSI_X); f2_mul(&r->y, &y, &PSI_Y); r->z = z;
}
static void g2_psi2(g2j* r, const g2j* p) { f2_mul(&r->x, &p->x, &PSI2_X); f2_mul(&r->y, &p->y, &PSI2_Y); r->z = p->z; }
static void g2_mul_x(g2j* r, const g2j* p) { /* [x]P, x < 0 */
  g2_mul_u64(r, p, XABS);
  f2_neg(&r->y, &r->y);
}
static int g2_in_group(const g2j* p) {
  if (f2_is_zero(&p->z)) return 1;
  g2j a, b;
  g2_psi(&a, p);
  g2_mul_x(&b, p);
  return g2_eq(&a, &b);
}

/* ---------------------------------------------------------- encodings */
enum { OK = 0, BAD_ENCODING = 1, NOT_ON_CURVE = 2, NOT_IN_GROUP = 3, PK_IS_INFINITY = 6, INVALID_SIZE = 8 };

static int plain_lt_p(const fp* a) { return !geq_p(a->l); }
static int g2_decode(g2a* out, const uint8_t* b, int len) {
  memset(out, 0, sizeof *out);
  if (len != 96 && len != 192) return INVALID_SIZE;
  uint8_t b0 = b[0];
  if (len == 96) {
    if (!(b0 & 0x80)) return BAD_ENCODING;
    if (b0 & 0x40) {
      int z = (b0 & 0x3f) == 0;
      for (int i = 1; i < 96; i++) z &= b[i] == 0;
      if (!z) return BAD_ENCODING;
      out->inf = 1;
      return OK;
    }
    uint8_t t[48];
    memcpy(t, b, 48);
    t[0] &= 0x1f;
    fp x1, x0;
    fp_from_be(&x1, t);
    fp_from_be(&x0, b + 48);
    if (!plain_lt_p(&x1) || !plain_lt_p(&x0)) return BAD_ENCODING;
    fp2 x, y2, y;
    to_mont(&x.c0, &x0);
    to_mont(&x.c1, &x1);
    f2_sqr(&y2, &x); f2_mul(&y2, &y2, &x); f2_add(&y2, &y2, &B2M);
    if (!f2_sqrt(&y, &y2)) return NOT_ON_CURVE;
    if (f2_lex(&y) != ((b0 & 0x20) != 0)) f2_neg(&y, &y);
    out->x = x;
    out->y = y;
    return OK;
  }
  if (b0 & 0x80) return BAD_ENCODING;
  if (b0 & 0x40) {
    int z = (b0 & 0x3f) == 0;
    for (int i = 1; i < 192; i++) z &= b[i] == 0;
    if (!z) return BAD_ENCODING;
    out->inf = 1;
    return OK;
  }
  if (b0 & 0x20) return BAD_ENCODING; /* a sign bit only exists on compressed encodings */
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  fp v[4];
  fp_from_be(&v[0], t);
  fp_from_be(&v[1], b + 48);
  fp_from_be(&v[2], b + 96);
  fp_from_be(&v[3], b + 144);
  for (int i = 0; i < 4; i++)
    if (!plain_lt_p(&v[i])) return BAD_ENCODING;
  to_mont(&out->x.c1, &v[0]); to_mont(&out->x.c0, &v[1]); to_mont(&out->y.c1, &v[2]); to_mont(&out->y.c0, &v[3]);
  fp2 l, r;
  f2_sqr(&l, &out->y);
  f2_sqr(&r, &out->x); f2_mul(&r, &r, &out->x); f2_add(&r, &r, &B2M);
  if (!f2_eq(&l, &r)) return NOT_ON_CURVE;
  return OK;
}
static int sig_from_bytes(g2a* out, const uint8_t* b, int len) {
  int c = g2_decode(out, b, len);
  if (c) return c;
  if (!out->inf) {
    g2j j;
    g2_from_aff(&j, out);
    if (!g2_in_group(&j)) return NOT_IN_GROUP;
  }
  return OK;
}
static int g1_decode96(g1a* out, const uint8_t* b) { /* trusted uncompressed */
  memset(out, 0, sizeof *out);
  if (b[0] & 0x40) { out->inf = 1; return OK; }
  uint8_t t[48];
  memcpy(t, b, 48);
  t[0] &= 0x1f;
  fp x, y;
  fp_from_be(&x, t);
  fp_from_be(&y, b + 48);
  to_mont(&out->x, &x);
  to_mont(&out->y, &y);
  return OK;
}
static void g2_compress(uint8_t* out, const g2j* p) {
  g2a a;
  g2_to_aff(&a, p);
  memset(out, 0, 96);
  if (a.inf) { out[0] = 0xc0; return; }
  fp t;
  from_mont(&t, &a.x.c1); fp_to_be(out, &t);
  from_mont(&t, &a.x.c0); fp_to_be(out + 48, &t);
  out[0] |= 0x80 | (f2_lex(&a.y) ? 0x20 : 0);
}
static void g1_serialize(uint8_t* out, const g1j* p) {
  g1a a;
  g1_to_aff(&a, p);
  memset(out, 0, 96);
  if (a.inf) { out[0] = 0x40; return; }
  fp t;
  from_mont(&t, &a.x); fp_to_be(out, &t);
  from_mont(&t, &a.y); fp_to_be(out + 48, &t);
}

/* -------------------------------------------------------------- SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
    0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
    0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
    0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256(uint8_t out[32], const uint8_t* msg, size_t len) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t total = ((len + 9 + 63) / 64) * 64;
  uint8_t* buf = (uint8_t*)calloc(total, 1);
  memcpy(buf, msg, len);
  buf[len] = 0x80;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) buf[total - 1 - i] = (uint8_t)(bits >> (8 * i));
  for (size_t off = 0; off < total; off += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)buf[off + 4 * i] << 24 | (uint32_t)buf[off + 4 * i + 1] << 16 | (uint32_t)buf[off + 4 * i + 2] << 8 | buf[off + 4 * i + 3];
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
      uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  free(buf);
  for (int i = 0; i < 8; i++) for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
}

/* --------------------------------------------------------- hash to G2 */
static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
static void expand_xmd(uint8_t out[256], const uint8_t* msg, size_t mlen) {
  const size_t dl = sizeof(DST) - 1;
  uint8_t dstp[64];
  memcpy(dstp, DST, dl);
  dstp[dl] = (uint8_t)dl;
  uint8_t buf[64 + 64 + 3 + 64];
  size_t n = 0;
  memset(buf, 0, 64);
  n = 64;
  memcpy(buf + n, msg, mlen); n += mlen;
  buf[n++] = 1; buf[n++] = 0; buf[n++] = 0;
  memcpy(buf + n, dstp, dl + 1); n += dl + 1;
  uint8_t b0[32], bi[32];
  sha256(b0, buf, n);
  for (int i = 1; i <= 8; i++) {
    uint8_t t[32 + 1 + 64];
    for (int k = 0; k < 32; k++) t[k] = (uint8_t)(b0[k] ^ (i == 1 ? 0 : bi[k]));
    t[32] = (uint8_t)i;
    memcpy(t + 33, dstp, dl + 1);
    sha256(bi, t, 33 + dl + 1);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}
static void fp_from_64be(fp* r, const uint8_t* b) { /* 64 bytes big-endian mod p */
  fp hi, lo, t;
  uint8_t x[48];
  memset(x, 0, 48);
  memcpy(x + 16, b, 32);
  fp_from_be(&hi, x);
  memcpy(x + 16, b + 32, 32);
  fp_from_be(&lo, x);
  /* hi * 2^256 + lo: to Montgomery, then multiply hi by 2^256 */
  to_mont(&hi, &hi);
  to_mont(&lo, &lo);
  fp_mul(&t, &hi, &T256);
  fp_add(r, &t, &lo);
}
/* simplified SWU onto E2' (RFC 9380 6.6.2) with the device's shortcut
 * (lodestar_amd/csrc/h2c.h map_to_curve_sswu): one exponentiation of
 * norm(gx1) answers the square test and starts the root; when gx1 is not a
 * square, sqrt(norm(gx2)) = sqrt(-norm(Z)^3) norm(u)^3 d. */
static fp SQRT_NEG_NZ3;
static void map_sswu(g2a* out, const fp2* u) {
  fp2 u2, zu2, den, tv, x1, x2, gx1, gx2, t, x, g, y;
  f2_sqr(&u2, u);
  f2_mul(&zu2, &S_Z, &u2);
  f2_sqr(&den, &zu2);
  f2_add(&den, &den, &zu2);
  if (f2_is_zero(&den)) x1 = S_BZA;
  else {
    f2_inv(&tv, &den);
    fp_add(&tv.c0, &tv.c0, &FONE);
    f2_mul(&x1, &S_MBA, &tv);
  }
  f2_sqr(&t, &x1); f2_add(&t, &t, &S_A); f2_mul(&gx1, &t, &x1); f2_add(&gx1, &gx1, &S_B);
  f2_mul(&x2, &zu2, &x1);
  f2_sqr(&t, &x2); f2_add(&t, &t, &S_A); f2_mul(&gx2, &t, &x2); f2_add(&gx2, &gx2, &S_B);
  fp n1, d, chk, nu, nu3;
  f2_norm(&n1, &gx1);
  fp_pow(&d, &n1, &E_SQRT);
  fp_sqr(&chk, &d);
  const int sq = fp_eq(&chk, &n1);
  if (sq) { x = x1; g = gx1; }
  else {
    x = x2; g = gx2;
    f2_norm(&nu, u);
    fp_sqr(&nu3, &nu); fp_mul(&nu3, &nu3, &nu);
    fp_mul(&d, &d, &nu3);
    fp_mul(&d, &d, &SQRT_NEG_NZ3);
  }
  if (fp_is_zero(&g.c1) || (!sq && f2_is_zero(&den))) f2_sqrt(&y, &g);
  else f2_sqrt_tail(&y, &g, &d);
  if (f2_sgn0(u) != f2_sgn0(&y)) f2_neg(&y, &y);
  out->x = x; out->y = y; out->inf = 0;
}
static void horner(fp2* r, const fp2* c, int n, const fp2* x) {
  fp2 acc = c[n - 1];
  for (int i = n - 2; i >= 0; i--) { f2_mul(&acc, &acc, x); f2_add(&acc, &acc, &c[i]); }
  *r = acc;
}
static void iso_map(g2j* r, const g2a* p) {
  fp2 xn, xd, yn, yd, t, yd2;
  horner(&xn, IXN, 4, &p->x); horner(&xd, IXD, 3, &p->x); horner(&yn, IYN, 4, &p->x); horner(&yd, IYD, 4, &p->x);
  f2_mul(&r->z, &xd, &yd);
  f2_sqr(&yd2, &yd);
  f2_mul(&t, &xn, &xd); f2_mul(&r->x, &t, &yd2);
  f2_sqr(&t, &xd); f2_mul(&t, &t, &xd); f2_mul(&t, &t, &yd2); f2_mul(&t, &t, &yn); f2_mul(&r->y, &t, &p->y);
}
static void clear_cofactor(g2j* r, const g2j* p) {
  g2j t1, t2, t3, np;
  g2_mul_x(&t1, p);
  g2_mul_x(&t2, &t1);
  np = *p; f2_neg(&np.y, &np.y);
  g2j_add(&t3, &t1, &np); g2_psi(&t3, &t3);
  f2_neg(&t1.y, &t1.y);
  g2j_add(&t2, &t2, &t1); g2j_add(&t2, &t2, &np); g2j_add(&t2, &t2, &t3);
  g2j_dbl(&t1, p); g2_psi2(&t1, &t1);
  g2j_add(r, &t2, &t1);
}
static void hash_to_g2(g2j* r, const uint8_t* msg, size_t len) {
  uint8_t ub[256];
  expand_xmd(ub, msg, len);
  fp2 u0, u1;
  fp_from_64be(&u0.c0, ub); fp_from_64be(&u0.c1, ub + 64); fp_from_64be(&u1.c0, ub + 128); fp_from_64be(&u1.c1, ub + 192);
  g2a q0, q1;
  map_sswu(&q0, &u0);
  map_sswu(&q1, &u1);
  g2j j0, j1, s;
  iso_map(&j0, &q0);
  iso_map(&j1, &q1);
  g2j_add(&s, &j0, &j1);
  clear_cofactor(r, &s);
}

/* ------------------------------------------------------------- pairing */
typedef struct { fp2 x, y, z; } g2p;
static void dbl_step(g2p* T, fp2* a0, fp2* a1, fp2* b1, const g1a* P) {
  fp2 A, B, C, E, F, G, H, t;
  f2_mul(&A, &T->x, &T->y); fp_mul(&A.c0, &A.c0, &FHALF); fp_mul(&A.c1, &A.c1, &FHALF);
  f2_sqr(&B, &T->y); f2_sqr(&C, &T->z); f2_mul(&E, &C, &B2X3);
  f2_add(&F, &E, &E); f2_add(&F, &F, &E);
  f2_add(&t, &T->y, &T->z); f2_sqr(&t, &t); f2_add(&H, &B, &C); f2_sub(&H, &t, &H);
  f2_sub(a0, &E, &B);
  f2_sqr(&t, &T->x); fp2 t3; f2_add(&t3, &t, &t); f2_add(&t3, &t3, &t); f2_mul_fp(a1, &t3, &P->x);
  f2_mul_fp(&t, &H, &P->y); f2_neg(b1, &t);
  f2_sub(&t, &B, &F); f2_mul(&T->x, &A, &t);
  f2_add(&G, &B, &F); fp_mul(&G.c0, &G.c0, &FHALF); fp_mul(&G.c1, &G.c1, &FHALF); f2_sqr(&G, &G);
  f2_sqr(&t, &E); f2_add(&t3, &t, &t); f2_add(&t3, &t3, &t); f2_sub(&T->y, &G, &t3);
  f2_mul(&T->z, &B, &H);
}
static void add_step(g2p* T, fp2* a0, fp2* a1, fp2* b1, const g2a* Q, const g1a* P) {
  fp2 th, la, C, D, E, F, G, H, t;
  f2_mul(&t, &Q->y, &T->z); f2_sub(&th, &T->y, &t);
  f2_mul(&t, &Q->x, &T->z); f2_sub(&la, &T->x, &t);
  f2_mul(a0, &th, &Q->x); f2_mul(&t, &la, &Q->y); f2_sub(a0, a0, &t);
  f2_mul_fp(&t, &th, &P->x); f2_neg(a1, &t);
  f2_mul_fp(b1, &la, &P->y);
  f2_sqr(&C, &th); f2_sqr(&D, &la); f2_mul(&E, &D, &la); f2_mul(&F, &T->z, &C); f2_mul(&G, &T->x, &D);
  f2_add(&H, &E, &F); f2_sub(&H, &H, &G); f2_sub(&H, &H, &G);
  f2_mul(&T->x, &la, &H); f2_sub(&t, &G, &H); f2_mul(&t, &th, &t); f2_mul(&C, &T->y, &E); f2_sub(&T->y, &t, &C);
  f2_mul(&T->z, &T->z, &E);
}
/* multi-Miller loop over n pairs with one shared accumulator (x < 0: conjugate) */
static void miller_multi(fp12* f, const g1a* P, const g2a* Q, int n) {
  f12_one(f);
  g2p* T = (g2p*)malloc(sizeof(g2p) * (n ? n : 1));
  for (int k = 0; k < n; k++) { T[k].x = Q[k].x; T[k].y = Q[k].y; memset(&T[k].z, 0, sizeof(fp2)); T[k].z.c0 = FONE; }
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f12_sqr(f, f);
    for (int k = 0; k < n; k++) {
      if (P[k].inf || Q[k].inf) continue;
      fp2 a0, a1, b1;
      dbl_step(&T[k], &a0, &a1, &b1, &P[k]);
      f12_mul_line(f, &a0, &a1, &b1);
    }
    if ((XABS >> b) & 1)
      for (int k = 0; k < n; k++) {
        if (P[k].inf || Q[k].inf) continue;
        fp2 a0, a1, b1;
        add_step(&T[k], &a0, &a1, &b1, &Q[k], &P[k]);
        f12_mul_line(f, &a0, &a1, &b1);
      }
  }
  f12_conj(f, f);
  free(T);
}

/* --------------------------------------------------------------- init */
static void hex2(fp2* r, const char* const h[2]) { hex_to_fp(&r->c0, h[0]); hex_to_fp(&r->c1, h[1]); }
static void exp_consts(void) {
  /* E_PM2 = p - 2, E_SQRT = (p + 1) / 4, E_LEG = (p - 1) / 2, E_P34 = (p - 3) / 4 (plain) */
  memcpy(E_PM2.l, PM, 48); E_PM2.l[0] -= 2;
  uint64_t t[6];
  memcpy(t, PM, 48); t[0] += 1; /* p + 1 (no carry: low limb ends ...aaab) */
  for (int i = 0; i < 6; i++) E_SQRT.l[i] = (t[i] >> 2) | (i < 5 ? t[i + 1] << 62 : 0);
  memcpy(t, PM, 48); t[0] -= 1;
  for (int i = 0; i < 6; i++) E_LEG.l[i] = (t[i] >> 1) | (i < 5 ? t[i + 1] << 63 : 0);
  memcpy(t, PM, 48); t[0] -= 3;
  for (int i = 0; i < 6; i++) E_P34.l[i] = (t[i] >> 2) | (i < 5 ? t[i + 1] << 62 : 0);
}
void bref_init(void) {
  if (inited) return;
  memcpy(PMX, PM, 48);
  PMX[6] = PINV;
  __builtin_cpu_init();
  use_mulx = __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx");
  /* R mod p and R^2 mod p by doubling (plain arithmetic mod p via fp_add) */
  fp one;
  memset(&one, 0, sizeof one);
  one.l[0] = 1;
  fp x = one;
  for (int i = 0; i < 384; i++) fp_add(&x, &x, &x);
  R1 = x;
  for (int i = 0; i < 384; i++) fp_add(&x, &x, &x);
  R2 = x;
  FONE = R1;
  memcpy(PMX, PM, 48);
  PMX[6] = PINV;
  fp_mul(&R3, &R2, &R2);
  exp_consts();
  fp two = FONE;
  fp_add(&two, &two, &two);
  fp_inv(&FHALF, &two);
  fp four = two;
  fp_add(&four, &four, &four);
  B2M.c0 = four;
  B2M.c1 = four;
  fp2 t3;
  f2_add(&t3, &B2M, &B2M);
  f2_add(&B2X3, &t3, &B2M);
  hex_to_fp(&G1A.x, C_G1[0]);
  hex_to_fp(&G1A.y, C_G1[1]);
  G1A.inf = 0;
  G1NEG = G1A;
  fp_neg(&G1NEG.y, &G1NEG.y);
  hex2(&G2X, C_G2[0]);
  hex2(&G2Y, C_G2[1]);
  hex2(&PSI_X, C_PSI[0]); hex2(&PSI_Y, C_PSI[1]);
  hex2(&PSI2_X, C_PSI2[0]); hex2(&PSI2_Y, C_PSI2[1]);
  for (int k = 0; k < 3; k++) for (int i = 0; i < 5; i++) hex2(&FROB[k][i], C_FROB[5 * k + i]);
  hex2(&S_A, C_SSWU[0]); hex2(&S_B, C_SSWU[1]); hex2(&S_Z, C_SSWU[2]);
  for (int i = 0; i < 4; i++) { hex2(&IXN[i], C_ISO_XNUM[i]); hex2(&IYN[i], C_ISO_YNUM[i]); hex2(&IYD[i], C_ISO_YDEN[i]); }
  for (int i = 0; i < 3; i++) hex2(&IXD[i], C_ISO_XDEN[i]);
  /* -B/A and B/(Z A) */
  fp2 ia, t;
  f2_inv(&ia, &S_A);
  f2_mul(&t, &S_B, &ia); f2_neg(&S_MBA, &t);
  f2_mul(&t, &S_Z, &S_A); f2_inv(&t, &t); f2_mul(&S_BZA, &S_B, &t);
  {
    fp nz, nz3;
    f2_norm(&nz, &S_Z);
    fp_sqr(&nz3, &nz); fp_mul(&nz3, &nz3, &nz); fp_neg(&nz3, &nz3);
    fp_sqrt(&SQRT_NEG_NZ3, &nz3); /* -norm(Z)^3 is a square */
  }
  T256 = FONE;
  for (int i = 0; i < 256; i++) fp_add(&T256, &T256, &T256); /* 2^256, Montgomery */
  inited = 1;
}

/* ------------------------------------------------------------ exported API */
/* maybeBatch semantics for one job of n sets (pk = aggregated, 96 B uncompressed).
 * returns 1 valid, 0 invalid, -code on a parse error / infinity pk. */
static int verify_job_parsed(const g1a* pks, const uint8_t* msgs, const g2a* sigs, int n, const uint64_t* scalars) {
  for (int i = 0; i < n; i++)
    if (pks[i].inf) return -PK_IS_INFINITY;
  g1a* P = (g1a*)malloc(sizeof(g1a) * (n + 1));
  g2a* Q = (g2a*)malloc(sizeof(g2a) * (n + 1));
  g2j S;
  g2_set_inf(&S);
  for (int i = 0; i < n; i++) {
    uint64_t r = n >= 2 ? scalars[i] : 1;
    g1j pj, rp;
    g1_from_aff(&pj, &pks[i]);
    if (r != 1) g1_mul_u64(&rp, &pj, r); else rp = pj;
    g1_to_aff(&P[i], &rp);
    g2j h;
    hash_to_g2(&h, msgs + 32 * i, 32);
    g2_to_aff(&Q[i], &h);
    if (!sigs[i].inf) {
      g2j sj, rs;
      g2_from_aff(&sj, &sigs[i]);
      if (r != 1) g2_mul_u64(&rs, &sj, r); else rs = sj;
      g2j_add(&S, &S, &rs);
    }
  }
  P[n] = G1NEG;
  g2_to_aff(&Q[n], &S);
  fp12 f, e;
  miller_multi(&f, P, Q, n + 1);
  final_exp(&e, &f);
  free(P);
  free(Q);
  return f12_is_one(&e) ? 1 : 0;
}

int bref_verify_job(const uint8_t* pks96, const uint8_t* msgs, const uint8_t* sigs192, const uint32_t* sig_len, int n,
                    const uint64_t* scalars) {
  bref_init();
  if (n == 0) return -10;
  g2a* S = (g2a*)malloc(sizeof(g2a) * n);
  g1a* K = (g1a*)malloc(sizeof(g1a) * n);
  int code = 0;
  for (int i = 0; i < n && !code; i++) code = sig_from_bytes(&S[i], sigs192 + 192 * i, (int)sig_len[i]);
  int res;
  if (code) res = -code;
  else {
    for (int i = 0; i < n; i++) g1_decode96(&K[i], pks96 + 96 * i);
    res = verify_job_parsed(K, msgs, S, n, scalars);
  }
  free(S);
  free(K);
  return res;
}

/* aggregate k uncompressed pubkeys -> 96 B uncompressed (PublicKey.aggregate) */
void bref_aggregate(const uint8_t* pks96, int k, uint8_t* out96) {
  bref_init();
  g1j acc;
  g1_set_inf(&acc);
  for (int i = 0; i < k; i++) {
    g1a a;
    g1_decode96(&a, pks96 + 96 * i);
    if (a.inf) continue;
    g1j_add_aff(&acc, &acc, &a.x, &a.y);
  }
  g1_serialize(out96, &acc);
}

/* sk (32 B big-endian, < r) -> pk 96 B uncompressed */
void bref_sk_to_pk(const uint8_t* sk32, uint8_t* out96) {
  bref_init();
  uint64_t k[4];
  for (int i = 0; i < 4; i++) { k[i] = 0; for (int b = 0; b < 8; b++) k[i] = (k[i] << 8) | sk32[24 - 8 * i + b]; }
  g1j g, p;
  g1_from_aff(&g, &G1A);
  g1_mul_words(&p, &g, k, 4);
  g1_serialize(out96, &p);
}

/* sign: sk (32 B big-endian) -> 96 B compressed signature on msg32 */
void bref_sign(const uint8_t* sk32, const uint8_t* msg32, uint8_t* out96) {
  bref_init();
  uint64_t k[4];
  for (int i = 0; i < 4; i++) { k[i] = 0; for (int b = 0; b < 8; b++) k[i] = (k[i] << 8) | sk32[24 - 8 * i + b]; }
  g2j h, s;
  hash_to_g2(&h, msg32, 32);
  g2_mul_words(&s, &h, k, 4);
  g2_compress(out96, &s);
}

void bref_hash_to_g2(const uint8_t* msg, int len, uint8_t* out192) {
  bref_init();
  g2j h;
  hash_to_g2(&h, msg, (size_t)len);
  g2a a;
  g2_to_aff(&a, &h);
  fp t;
  from_mont(&t, &a.x.c1); fp_to_be(out192, &t);
  from_mont(&t, &a.x.c0); fp_to_be(out192 + 48, &t);
  from_mont(&t, &a.y.c1); fp_to_be(out192 + 96, &t);
  from_mont(&t, &a.y.c0); fp_to_be(out192 + 144, &t);
}

/* ---------------------------------------------------- threaded CPU bench */
/* jobs as in bgv_batch: job_off[J+1], pk_off[n+1], pk_idx into table96,
 * msgs[n][32], sigs[n][192], sig_len[n].  Each thread takes whole jobs
 * (the pool sends <= 128 sets per job to one worker) and does the
 * aggregation + maybeBatch verification.  Writes job results. */
typedef struct {
  const uint32_t *job_off, *pk_off, *pk_idx, *sig_len;
  const uint8_t *table96, *msgs, *sigs;
  int n_jobs;
  int* results;
  volatile int next;
  pthread_mutex_t mu;
  uint64_t seed;
} bench_ctx;

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static void* bench_worker(void* arg) {
  bench_ctx* c = (bench_ctx*)arg;
  for (;;) {
    pthread_mutex_lock(&c->mu);
    int j = c->next++;
    pthread_mutex_unlock(&c->mu);
    if (j >= c->n_jobs) break;
    uint32_t beg = c->job_off[j], end = c->job_off[j + 1];
    int n = (int)(end - beg);
    g1a* K = (g1a*)malloc(sizeof(g1a) * (n ? n : 1));
    g2a* S = (g2a*)malloc(sizeof(g2a) * (n ? n : 1));
    uint64_t* r = (uint64_t*)malloc(8 * (n ? n : 1));
    uint64_t sd = c->seed ^ ((uint64_t)j << 32);
    int code = 0;
    for (int i = 0; i < n; i++) {
      r[i] = splitmix(&sd) | 1;
      /* main-thread aggregation of the reference (utils.ts:11), here in the worker */
      g1j acc;
      g1_set_inf(&acc);
      for (uint32_t k = c->pk_off[beg + i]; k < c->pk_off[beg + i + 1]; k++) {
        g1a a;
        g1_decode96(&a, c->table96 + 96ull * c->pk_idx[k]);
        if (!a.inf) g1j_add_aff(&acc, &acc, &a.x, &a.y);
      }
      g1_to_aff(&K[i], &acc);
      if (!code) code = sig_from_bytes(&S[i], c->sigs + 192ull * (beg + i), (int)c->sig_len[beg + i]);
    }
    c->results[j] = n == 0 ? -10 : code ? -code : verify_job_parsed(K, c->msgs + 32ull * beg, S, n, r);
    free(K);
    free(S);
    free(r);
  }
  return NULL;
}

/* returns wall seconds */
double bref_bench_jobs(const uint32_t* job_off, int n_jobs, const uint32_t* pk_off, const uint32_t* pk_idx,
                       const uint8_t* table96, const uint8_t* msgs, const uint8_t* sigs, const uint32_t* sig_len,
                       int threads, int* results) {
  bref_init();
  bench_ctx c;
  memset(&c, 0, sizeof c);
  c.job_off = job_off; c.pk_off = pk_off; c.pk_idx = pk_idx; c.sig_len = sig_len;
  c.table96 = table96; c.msgs = msgs; c.sigs = sigs; c.n_jobs = n_jobs; c.results = results;
  c.seed = 0x1234;
  pthread_mutex_init(&c.mu, NULL);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, bench_worker, &c);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  pthread_mutex_destroy(&c.mu);
  return (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
}
