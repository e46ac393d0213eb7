// Host-compiled view of the device arithmetic headers (lodestar_amd/csrc/*.h)
// for CPU-side debugging tests against the Python oracle.  TEST ONLY: the
// product never executes this; it launches the HIP kernels through libbgv.
// I/O convention: Fp = 48-byte big-endian plain integer; Fp2 = c0 || c1;
// affine G2 = x || y (192 B); affine G1 = x || y (96 B); Fp12 = 12 Fp
// coefficients ordered w^0.c0, w^0.c1, w^1.c0, ... (tower position k at w^k).
#include <string.h>
#include "../../lodestar_amd/csrc/pairing.h"
#include "../../lodestar_amd/csrc/rng.h"

using namespace bgv;

static void get_fp(fp_t& r, const uint8_t* b) { fp_t t; fp_from_be48(t, b); fp_to_mont(r, t); }
static void put_fp(uint8_t* b, const fp_t& a) { fp_t t; fp_from_mont(t, a); fp_to_be48(b, t); }
static void get_fp2(fp2_t& r, const uint8_t* b) { get_fp(r.c0, b); get_fp(r.c1, b + 48); }
static void put_fp2(uint8_t* b, const fp2_t& a) { put_fp(b, a.c0); put_fp(b + 48, a.c1); }
static void get_g2a(g2a& r, const uint8_t* b) { get_fp2(r.x, b); get_fp2(r.y, b + 96); }
static void put_g2a(uint8_t* b, const g2a& a) { put_fp2(b, a.x); put_fp2(b + 96, a.y); }
static void get_g1a(g1a& r, const uint8_t* b) { get_fp(r.x, b); get_fp(r.y, b + 48); }
static void put_g1a(uint8_t* b, const g1a& a) { put_fp(b, a.x); put_fp(b + 48, a.y); }
static void put_fp12(uint8_t* b, const fp12_t& f) {
  const fp2_t* c[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  for (int k = 0; k < 6; k++) put_fp2(b + 96 * k, *c[k]);
}
static void get_fp12(fp12_t& f, const uint8_t* b) {
  fp2_t* c[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  for (int k = 0; k < 6; k++) get_fp2(*c[k], b + 96 * k);
}
// Jacobian -> affine bytes; returns 0 for infinity
static int put_g2j(uint8_t* b, const g2j& p) { g2a a; bool ok = jac_to_aff(a, p); put_g2a(b, a); return ok; }
static int put_g1j(uint8_t* b, const g1j& p) { g1a a; bool ok = jac_to_aff(a, p); put_g1a(b, a); return ok; }

extern "C" {

void hc_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp_t x, y, z; get_fp(x, a); get_fp(y, b); fp_mul(z, x, y); put_fp(out, z); }
void hc_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp_t x, y, z; get_fp(x, a); get_fp(y, b); fp_add(z, x, y); put_fp(out, z); }
void hc_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp_t x, y, z; get_fp(x, a); get_fp(y, b); fp_sub(z, x, y); put_fp(out, z); }
void hc_fp_inv(const uint8_t* a, uint8_t* out) { fp_t x, z; get_fp(x, a); fp_inv(z, x); put_fp(out, z); }
void hc_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp2_t x, y, z; get_fp2(x, a); get_fp2(y, b); fp2_mul(z, x, y); put_fp2(out, z); }
void hc_fp2_sqr(const uint8_t* a, uint8_t* out) { fp2_t x, z; get_fp2(x, a); fp2_sqr(z, x); put_fp2(out, z); }
void hc_fp2_inv(const uint8_t* a, uint8_t* out) { fp2_t x, z; get_fp2(x, a); fp2_inv(z, x); put_fp2(out, z); }
// fp_mul on unreduced inputs a + p, b + p (< 2p, the fp_add_lazy range) must
// return the same canonical limbs as on a, b; returns the number of failures
void hc_fp2_mul_sop(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  fp2_t x, y, z; get_fp2(x, a); get_fp2(y, b); fp2_mul_sop(z, x, y); put_fp2(out, z);
}

// the sum-of-products Fp2 product (fp2_mul_sop, the device's Fp2 leaf) against
// Karatsuba on canonical operands and on lazy ones (x + p < 2p in any
// component, and the extremes p - 1, 2p - 1): bit-identical canonical output
int hc_sop_lazy_check(uint64_t seed, int n) {
  uint64_t x = seed | 1;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  auto canon = [&](fp_t& a) {
    for (int i = 0; i < NL; i++) a.l[i] = (uint32_t)rnd();
    a.l[NL - 1] &= 0x1fffffffu;
    fp_reduce_once(a, a); fp_reduce_once(a, a);
    if (!fp_plain_lt_p(a)) fp_sub(a, a, P_MOD);
  };
  auto lazy = [&](fp_t& r, const fp_t& a) {
    uint64_t c = 0;
    for (int i = 0; i < NL; i++) { c += (uint64_t)a.l[i] + P_MOD.l[i]; r.l[i] = (uint32_t)c; c >>= 32; }
  };
  int bad = 0;
  for (int it = 0; it < n; it++) {
    fp2_t a, b;
    canon(a.c0); canon(a.c1); canon(b.c0); canon(b.c1);
    if (it < 4) { a.c1 = P_MOD; a.c1.l[0] -= 1; b.c1 = a.c1; }  // p - 1
    if (it == 1) fp_set_zero(a.c1);
    fp2_t k, s, al, bl, sl;
    const uint32_t sel = (uint32_t)rnd();
    al = a; bl = b;
    if (sel & 1) lazy(al.c0, a.c0);
    if (sel & 2) lazy(al.c1, a.c1);
    if (sel & 4) lazy(bl.c0, b.c0);
    if (sel & 8) lazy(bl.c1, b.c1);
    if (it == 2) { lazy(al.c0, a.c0); lazy(al.c1, a.c1); lazy(bl.c0, b.c0); lazy(bl.c1, b.c1); }  // 2p - 1 everywhere
    // Karatsuba on the canonical values (the host path of fp2_mul)
    fp_t t0, t1, t2, t3;
    fp_mul(t0, a.c0, b.c0); fp_mul(t1, a.c1, b.c1);
    fp_add_lazy2(t2, a.c0, a.c1, t3, b.c0, b.c1); fp_mul(t2, t2, t3);
    fp_sub2(k.c0, t0, t1, t2, t2, t0); fp_sub(k.c1, t2, t1);
    fp2_mul_sop(s, a, b);
    fp2_mul_sop(sl, al, bl);
    if (memcmp(&k, &s, sizeof k) || memcmp(&k, &sl, sizeof k)) bad++;
    if (!fp_plain_lt_p(sl.c0) || !fp_plain_lt_p(sl.c1)) bad++;
  }
  return bad;
}

int hc_lazy_mul_canonical(uint64_t seed, int n) {
  uint64_t x = seed | 1;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  int bad = 0;
  for (int it = 0; it < n; it++) {
    fp_t a, b;
    for (int i = 0; i < NL; i++) { a.l[i] = (uint32_t)rnd(); b.l[i] = (uint32_t)rnd(); }
    a.l[NL - 1] &= 0x1fffffffu; b.l[NL - 1] &= 0x1fffffffu;
    if (it < 3) { a = P_MOD; a.l[0] -= 1 + it; }  // p-1, p-2, p-3
    fp_reduce_once(a, a); fp_reduce_once(a, a); fp_reduce_once(b, b); fp_reduce_once(b, b);
    if (!fp_plain_lt_p(a)) fp_sub(a, a, P_MOD);
    if (!fp_plain_lt_p(b)) fp_sub(b, b, P_MOD);
    fp_t ap, bp, r1, r2, r3;
    uint64_t c = 0, d = 0;
    for (int i = 0; i < NL; i++) {
      c += (uint64_t)a.l[i] + P_MOD.l[i]; ap.l[i] = (uint32_t)c; c >>= 32;
      d += (uint64_t)b.l[i] + P_MOD.l[i]; bp.l[i] = (uint32_t)d; d >>= 32;
    }
    fp_mul(r1, ap, bp);
    fp_mul(r2, a, b);
    fp_mul(r3, ap, b);
    for (int i = 0; i < NL; i++) if (r1.l[i] != r2.l[i] || r3.l[i] != r2.l[i]) { bad++; break; }
    if (!fp_plain_lt_p(r1)) bad++;
    // dedicated squaring (fp_sqr28) against the product, canonical and lazy (< 2p) inputs
    fp_t s1, s2, s3;
    fp_mul28(s1, a, a);
    fp_sqr28(s2, a);
    fp_sqr28(s3, ap);
    for (int i = 0; i < NL; i++) if (s1.l[i] != s2.l[i] || s1.l[i] != s3.l[i]) { bad++; break; }
    if (!fp_plain_lt_p(s3)) bad++;
  }
  return bad;
}

int hc_fp2_sqrt(const uint8_t* a, uint8_t* out) { fp2_t x, z; get_fp2(x, a); int ok = fp2_sqrt(z, x); put_fp2(out, z); return ok; }
int hc_fp2_is_square(const uint8_t* a) { fp2_t x; get_fp2(x, a); return fp2_is_square(x); }
int hc_fp2_sgn0(const uint8_t* a) { fp2_t x; get_fp2(x, a); return (int)fp2_sgn0(x); }

void hc_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { fp12_t x, y, z; get_fp12(x, a); get_fp12(y, b); fp12_mul(z, x, y); put_fp12(out, z); }
void hc_fp12_sqr(const uint8_t* a, uint8_t* out) { fp12_t x, z; get_fp12(x, a); fp12_sqr(z, x); put_fp12(out, z); }
void hc_fp12_inv(const uint8_t* a, uint8_t* out) { fp12_t x, z; get_fp12(x, a); fp12_inv(z, x); put_fp12(out, z); }
void hc_fp12_frob(const uint8_t* a, int k, uint8_t* out) { fp12_t x, z; get_fp12(x, a); fp12_frob(z, x, k); put_fp12(out, z); }
void hc_fp12_cyc_sqr(const uint8_t* a, uint8_t* out) { fp12_t x, z; get_fp12(x, a); fp12_cyclotomic_sqr(z, x); put_fp12(out, z); }
void hc_fp12_final_exp(const uint8_t* a, uint8_t* out) { fp12_t x, z; get_fp12(x, a); fp12_final_exp(z, x); put_fp12(out, z); }
void hc_fp12_mul_line(const uint8_t* f, const uint8_t* a0, const uint8_t* a1, const uint8_t* b1, uint8_t* out) {
  fp12_t x, z; fp2_t l0, l1, l2; get_fp12(x, f); get_fp2(l0, a0); get_fp2(l1, a1); get_fp2(l2, b1);
  fp12_mul_line(z, x, l0, l1, l2); put_fp12(out, z);
}

int hc_g2_decompress(const uint8_t* in96, uint8_t* out192, int* inf) {
  g2a a; bool i; int code = g2_decompress(a, i, in96); *inf = i; if (code == 0) put_g2a(out192, a); return code;
}
int hc_g2_deserialize(const uint8_t* in192, uint8_t* out192, int* inf) {
  g2a a; bool i; int code = g2_deserialize(a, i, in192); *inf = i; if (code == 0) put_g2a(out192, a); return code;
}
int hc_g1_decompress(const uint8_t* in48, uint8_t* out96, int* inf) {
  g1a a; bool i; int code = g1_decompress(a, i, in48); *inf = i; if (code == 0) put_g1a(out96, a); return code;
}
int hc_g2_in_subgroup(const uint8_t* aff192) { g2a a; get_g2a(a, aff192); g2j j; jac_from_aff(j, a); return g2_in_subgroup(j); }
int hc_g2_mul_u64(const uint8_t* aff192, uint64_t k, uint8_t* out192) { g2a a; get_g2a(a, aff192); g2j j, r; jac_from_aff(j, a); jac_mul_u64(r, j, k); return put_g2j(out192, r); }
int hc_g2_mul_u64_w4(const uint8_t* aff192, uint64_t k, uint8_t* out192) { g2a a; get_g2a(a, aff192); g2j j, r; jac_from_aff(j, a); jac_mul_u64_w4(r, j, k); return put_g2j(out192, r); }
int hc_g1_mul_u64_w4(const uint8_t* aff96, uint64_t k, uint8_t* out96) { g1a a; get_g1a(a, aff96); g1j j, r; jac_from_aff(j, a); jac_mul_u64_w4(r, j, k); return put_g1j(out96, r); }
int hc_g1_mul_u64(const uint8_t* aff96, uint64_t k, uint8_t* out96) { g1a a; get_g1a(a, aff96); g1j j, r; jac_from_aff(j, a); jac_mul_u64(r, j, k); return put_g1j(out96, r); }
int hc_g2_add(const uint8_t* a192, const uint8_t* b192, uint8_t* out192) {
  g2a a, b; get_g2a(a, a192); get_g2a(b, b192); g2j ja, jb, r; jac_from_aff(ja, a); jac_from_aff(jb, b); jac_add(r, ja, jb); return put_g2j(out192, r);
}
int hc_g2_dbl(const uint8_t* a192, uint8_t* out192) { g2a a; get_g2a(a, a192); g2j ja, r; jac_from_aff(ja, a); jac_dbl(r, ja); return put_g2j(out192, r); }
int hc_g1_sum(const uint8_t* pts96, int n, uint8_t* out96) {
  g1j acc; jac_set_inf(acc);
  for (int i = 0; i < n; i++) { g1a a; get_g1a(a, pts96 + 96 * i); jac_add_aff(acc, acc, a); }
  return put_g1j(out96, acc);
}
int hc_clear_cofactor(const uint8_t* aff192, uint8_t* out192) { g2a a; get_g2a(a, aff192); g2j j, r; jac_from_aff(j, a); g2_clear_cofactor(r, j); return put_g2j(out192, r); }

void hc_expand_message(const uint8_t* msg32, uint8_t* out256) {
  uint32_t w[64]; expand_message_xmd_256(w, msg32);
  for (int i = 0; i < 64; i++) { out256[4*i] = w[i] >> 24; out256[4*i+1] = w[i] >> 16; out256[4*i+2] = w[i] >> 8; out256[4*i+3] = w[i]; }
}
void hc_hash_to_field(const uint8_t* msg32, uint8_t* out384) { fp2_t u0, u1; hash_to_field_fp2x2(u0, u1, msg32); put_fp2(out384, u0); put_fp2(out384 + 192 - 96, u1); }
void hc_sswu(const uint8_t* u96, uint8_t* out192) { fp2_t u; get_fp2(u, u96); g2a q; map_to_curve_sswu(q, u); put_g2a(out192, q); }
int hc_iso_map(const uint8_t* aff192, uint8_t* out192) { g2a a; get_g2a(a, aff192); g2j r; iso_map_g2(r, a); return put_g2j(out192, r); }
int hc_hash_to_g2(const uint8_t* msg32, uint8_t* out192) { g2j r; hash_to_g2(r, msg32); return put_g2j(out192, r); }

void hc_miller_loop(const uint8_t* p96, const uint8_t* q192, uint8_t* out576) {
  g1a p; g2a q; get_g1a(p, p96); get_g2a(q, q192); fp12_t f; miller_loop(f, p, false, q, false); put_fp12(out576, f);
}
void hc_miller_loop2(const uint8_t* p1, const uint8_t* q1, const uint8_t* p2, const uint8_t* q2, uint8_t* out576) {
  g1a P1, P2; g2a Q1, Q2; get_g1a(P1, p1); get_g2a(Q1, q1); get_g1a(P2, p2); get_g2a(Q2, q2);
  fp12_t f; miller_loop2(f, P1, Q1, P2, Q2); put_fp12(out576, f);
}
void hc_miller_dbl_step(const uint8_t* t288, const uint8_t* p96, uint8_t* t_out288, uint8_t* line288) {
  g2p_t T; get_fp2(T.x, t288); get_fp2(T.y, t288 + 96); get_fp2(T.z, t288 + 192);
  g1a p; get_g1a(p, p96); fp2_t a0, a1, b1;
  miller_dbl_step(T, a0, a1, b1, p.x, p.y);
  put_fp2(t_out288, T.x); put_fp2(t_out288 + 96, T.y); put_fp2(t_out288 + 192, T.z);
  put_fp2(line288, a0); put_fp2(line288 + 96, a1); put_fp2(line288 + 192, b1);
}
void hc_miller_add_step(const uint8_t* t288, const uint8_t* q192, const uint8_t* p96, uint8_t* t_out288, uint8_t* line288) {
  g2p_t T; get_fp2(T.x, t288); get_fp2(T.y, t288 + 96); get_fp2(T.z, t288 + 192);
  g2a q; get_g2a(q, q192); g1a p; get_g1a(p, p96); fp2_t a0, a1, b1;
  miller_add_step(T, a0, a1, b1, q, p.x, p.y);
  put_fp2(t_out288, T.x); put_fp2(t_out288 + 96, T.y); put_fp2(t_out288 + 192, T.z);
  put_fp2(line288, a0); put_fp2(line288 + 96, a1); put_fp2(line288 + 192, b1);
}
}

extern "C" {
// ChaCha20 block function of the device scalar generator (rng.h)
void hc_chacha20_block(const uint32_t* key, uint32_t counter, const uint32_t* nonce, uint32_t* out) {
  chacha20_block(out, key, counter, nonce);
}
// split hash_to_G2 (two map lanes + finish) equals the one-lane hash_to_g2
int hc_hash_to_g2_split_eq(const uint8_t* msg) {
  g2j a, b, q0, q1;
  hash_to_g2(a, msg);
  hash_to_g2_map(q0, msg, 0);
  hash_to_g2_map(q1, msg, 1);
  hash_to_g2_finish(b, q0, q1);
  return jac_eq(a, b) ? 1 : 0;
}
}
