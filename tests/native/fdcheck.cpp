// Host build of the signed-digit field (lodestar_amd/csrc/fd.h) and of the
// latency kernels' cooperative G2 formulas (coop_g2_fd.h, one lane at a
// time through gd_host) with every fd bound asserted (-DBGV_FD_CHECK: a
// violated bound aborts).  TEST ONLY.  I/O as tests/native/hostcheck.cpp.
#include <string.h>
#include "../../lodestar_amd/csrc/coop_g2_fd.h"

using namespace bgv;

static void get_fp(fp_t& r, const uint8_t* b) { fp_t t; fp_from_be48(t, b); fp_to_mont(r, t); }
static void put_fp(uint8_t* b, const fp_t& a) { fp_t t; fp_from_mont(t, a); fp_to_be48(b, t); }
static void get_fp2(fp2_t& r, const uint8_t* b) { get_fp(r.c0, b); get_fp(r.c1, b + 48); }
static void put_fp2(uint8_t* b, const fp2_t& a) { put_fp(b, a.c0); put_fp(b + 48, a.c1); }
static void get_g2a(g2a& r, const uint8_t* b) { get_fp2(r.x, b); get_fp2(r.y, b + 96); }
static void put_g2a(uint8_t* b, const g2a& a) { put_fp2(b, a.x); put_fp2(b + 96, a.y); }
static int put_gd(uint8_t* b, const gd2j& p) {
  gd_host h;
  g2j j;
  gd_to_g2j(h, j, p);
  g2a a;
  const bool ok = jac_to_aff(a, j);
  put_g2a(b, a);
  return ok;
}
static void get_gd(gd2j& r, const uint8_t* b) { g2a a; get_g2a(a, b); gd_host h; gd_from_g2a(h, r, a); }

extern "C" {

void fdc_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  fp_t x, y, z; get_fp(x, a); get_fp(y, b);
  fd_t u, v, w; fd_from_fp(u, x); fd_from_fp(v, y); fd_mul(w, u, v); fd_to_fp(z, w); put_fp(out, z);
}
void fdc_sqr(const uint8_t* a, uint8_t* out) {
  fp_t x, z; get_fp(x, a);
  fd_t u, w; fd_from_fp(u, x); fd_sqr(w, u); fd_to_fp(z, w); put_fp(out, z);
}
// ((a + b)(a - 3c) - 2 (b - c)^2) / 2, with lazy digit sums, a norm, a fold,
// the halving and the zero test; returns is_zero(result - result)
int fdc_expr(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out) {
  fp_t x, y, z, r; get_fp(x, a); get_fp(y, b); get_fp(z, c);
  fd_t A, B, C, s, d, t, u, e, f;
  fd_from_fp(A, x); fd_from_fp(B, y); fd_from_fp(C, z);
  fd_add(s, A, B);
  fd_mulc<3>(t, C); fd_sub(d, A, t);
  fd_mul(u, s, d);
  fd_sub(t, B, C); fd_sqr(e, t);
  fd_dbl(e, e); fd_sub(f, u, e); fd_norm(f, f); fd_half(f, f); fd_fold(f, f);
  fd_to_fp(r, f); put_fp(out, r);
  fd_t zz; fd_sub(zz, f, f);
  return fd_is_zero(zz) && (fd_is_zero(f) == (fd_is_zero(A) && false ? true : fd_is_zero(f)));
}
int fdc_is_zero(const uint8_t* a) { fp_t x; get_fp(x, a); fd_t u; fd_from_fp(u, x); return fd_is_zero(u); }

int fdc_g2_dbl(const uint8_t* a192, uint8_t* out192) { gd2j p, r; get_gd(p, a192); gd_host h; gd_dbl(h, r, p); return put_gd(out192, r); }
int fdc_g2_add(const uint8_t* a192, const uint8_t* b192, uint8_t* out192) {
  gd2j p, q, r; get_gd(p, a192); get_gd(q, b192); gd_host h; gd_add(h, r, p, q); return put_gd(out192, r);
}
int fdc_g2_add_jac(const uint8_t* a192, const uint8_t* b192, uint8_t* out192) {
  // P as [2]P' (non-trivial z) plus Q, and P + P through the exceptional branch
  gd2j p, q, r, p2; get_gd(p, a192); get_gd(q, b192); gd_host h; gd_dbl(h, p2, p); gd_add(h, r, p2, q); return put_gd(out192, r);
}
int fdc_clear_cofactor(const uint8_t* a192, uint8_t* out192) { gd2j p, r; get_gd(p, a192); gd_host h; gd_clear_cofactor(h, r, p); return put_gd(out192, r); }
int fdc_in_subgroup(const uint8_t* a192) { gd2j p; get_gd(p, a192); gd_host h; return gd_in_subgroup(h, p); }
int fdc_mul_u64_w4(const uint8_t* a192, uint64_t k, uint8_t* out192) {
  gd2j p, r, tab[16]; get_gd(p, a192); gd_host h; gd_mul_u64_w4(h, tab, true, r, p, k); return put_gd(out192, r);
}
int fdc_mul_abs_x(const uint8_t* a192, uint8_t* out192) { gd2j p, r; get_gd(p, a192); gd_host h; gd_mul_abs_x(h, r, p); return put_gd(out192, r); }

}  // extern "C"
