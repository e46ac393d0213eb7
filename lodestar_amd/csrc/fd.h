// fd: a signed-digit, lazily reduced Fp for the latency kernels.
//
// A lone wave on CDNA4 issues one VALU instruction per ~4 cycles, and the
// 12 x 32-bit limb form of fp.h pays for its carries: every v_addc waits on
// the VCC written by the previous one (an s_nop per limb), so one reduced
// Fp addition costs 0.16 us against 0.98 us for a product
// (tools/ubench_lat.hip, profiles/r02_ubench_lat.json).  The cooperative
// kernels of the latency mode (coop_g2.h) run long chains of such additions
// between their product rounds.  Here an element is 14 SIGNED digits of
// radix 2^28,
//     v = sum_k d_k 2^(28 k),   Montgomery form with R = 2^392,
// and additions, subtractions and small multiples are digit-wise and
// carry-free (14 independent instructions, no VCC), so nothing is reduced
// until a product needs it.
//
// Bounds (checked on the host build, -DBGV_FD_CHECK, tests/native):
//   * the product (fd_mul / fd_sqr) accumulates 28 signed 64-bit columns of
//     up to 14 digit products and 14 reduction terms: it needs
//     max|a_k| max|b_k| <= 2^59 (e.g. 2^29.5 each), and its output value is
//     in (AB/R, AB/R + p): |out| <= 1.1 p whenever |A||B| <= 0.1 p R
//     (about (16 p)^2);
//   * every other operation keeps |digit| < 2^31;
//   * fd_norm re-normalizes the digits (values unchanged), fd_fold reduces
//     the value to |v| < 1.6 p.
// Products come out with digits 0..12 in [0, 2^28) and a small signed top
// digit ("normalized").
#pragma once
#include "fp.h"

namespace bgv {

constexpr int ND = 14;
constexpr int32_t FD_M = (1 << 28) - 1;
struct fd_t { int32_t d[ND]; };
struct fd2_t { fd_t c0, c1; };

}  // namespace bgv

#include "fd_consts.h"

#if !defined(__HIPCC__) && defined(BGV_FD_CHECK)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#define FD_ASSERT(c, msg)                                       \
  do {                                                          \
    if (!(c)) {                                                 \
      fprintf(stderr, "fd bound violated: %s (%s:%d)\n", msg, __FILE__, __LINE__); \
      abort();                                                  \
    }                                                           \
  } while (0)
#endif

namespace bgv {

#if !defined(__HIPCC__) && defined(BGV_FD_CHECK)
static inline double fd_value_abs(const fd_t& a) {
  double v = 0;
  for (int k = ND - 1; k >= 0; k--) v = v * 268435456.0 + (double)a.d[k];
  return std::fabs(v);
}
static inline double fd_digit_max(const fd_t& a) {
  double m = 0;
  for (int k = 0; k < ND; k++) m = std::fmax(m, std::fabs((double)a.d[k]));
  return m;
}
static inline void fd_check_mul(const fd_t& a, const fd_t& b) {
  FD_ASSERT(fd_digit_max(a) * fd_digit_max(b) <= 576460752303423488.0, "product digits > 2^59");
  const double p = 4.0024e114;  // p ~ 2^380.7
  FD_ASSERT(fd_value_abs(a) * fd_value_abs(b) <= 0.1 * p * std::ldexp(1.0, 392), "product values > 0.1 p R");
}
static inline int32_t fd_chk32(int64_t v) {
  FD_ASSERT(v > -2147483648LL && v < 2147483647LL, "digit overflows int32");
  return (int32_t)v;
}
#define FD_D(expr) fd_chk32((int64_t)(expr))
#else
#define FD_D(expr) (int32_t)(expr)
#endif

// ---- carry-free digit-wise operations ---------------------------------------
BGV_HD void fd_add(fd_t& r, const fd_t& a, const fd_t& b) {
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = FD_D((int64_t)a.d[k] + b.d[k]);
}
BGV_HD void fd_sub(fd_t& r, const fd_t& a, const fd_t& b) {
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = FD_D((int64_t)a.d[k] - b.d[k]);
}
BGV_HD void fd_neg(fd_t& r, const fd_t& a) {
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = -a.d[k];
}
template <int C> BGV_HD void fd_mulc(fd_t& r, const fd_t& a) {
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = FD_D((int64_t)a.d[k] * C);
}
BGV_HD void fd_dbl(fd_t& r, const fd_t& a) { fd_mulc<2>(r, a); }
BGV_HD void fd_zero(fd_t& r) {
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = 0;
}
BGV_HD void fd_select(fd_t& r, bool c, const fd_t& a, const fd_t& b) {
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = c ? a.d[k] : b.d[k];
}

// digits back to [0, 2^28) + a small carry (|d| < 2^31 in: |carry| <= 8);
// every output digit from two input digits, no chain
BGV_HD void fd_norm(fd_t& r, const fd_t& a) {
  fd_t t;
  t.d[0] = a.d[0] & FD_M;
#pragma unroll
  for (int k = 1; k < ND - 1; k++) t.d[k] = (a.d[k] & FD_M) + (a.d[k - 1] >> 28);
  t.d[ND - 1] = a.d[ND - 1] + (a.d[ND - 2] >> 28);
  r = t;
}

// value fold: v - q p with q = round(v / p) estimated from the top digit
// (digits normalized first); |result| < 1.6 p for |v| < 2^24 p
BGV_HD void fd_fold(fd_t& r, const fd_t& a_in) {
  fd_t a;
  fd_norm(a, a_in);
  const int32_t q = (int32_t)rintf((float)a.d[ND - 1] * FD_INV_PTOP);
  int64_t x[ND];
#pragma unroll
  for (int k = 0; k < ND; k++) x[k] = (int64_t)a.d[k] - (int64_t)q * FD_P28[k];
  r.d[0] = (int32_t)(x[0] & FD_M);
#pragma unroll
  for (int k = 1; k < ND - 1; k++) r.d[k] = (int32_t)((x[k] & FD_M) + (x[k - 1] >> 28));
  r.d[ND - 1] = FD_D(x[ND - 1] + (x[ND - 2] >> 28));
}

// v / 2 mod p: add p when v is odd (the parity of v is that of d_0), then a
// digit-wise shift that moves each digit's low bit down as 2^27
BGV_HD void fd_half(fd_t& r, const fd_t& a) {
  const int32_t odd = a.d[0] & 1;
  fd_t t;
#pragma unroll
  for (int k = 0; k < ND; k++) t.d[k] = FD_D((int64_t)a.d[k] + (odd ? FD_P28[k] : 0));
#pragma unroll
  for (int k = 0; k < ND - 1; k++) r.d[k] = (t.d[k] >> 1) + ((t.d[k + 1] & 1) << 27);
  r.d[ND - 1] = t.d[ND - 1] >> 1;
}

// ---- the product ------------------------------------------------------------
// Signed product scanning on 28 columns (v_mad_i64_i32), interleaved
// Montgomery reduction by 2^28 per digit (the reduction terms m p_j are
// non-negative; two's-complement addition makes the column sums exact).
BGV_HD void fd_mul_core(int32_t r[ND], const int32_t a[ND], const int32_t b[ND]) {
  uint64_t acc[2 * ND];
#pragma unroll
  for (int k = 0; k < 2 * ND; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < ND; i++)
#pragma unroll
    for (int j = 0; j < ND; j++) acc[i + j] += (uint64_t)((int64_t)a[i] * (int64_t)b[j]);
#pragma unroll
  for (int i = 0; i < ND; i++) {
    const uint32_t m = ((uint32_t)acc[i] * FD_PINV) & (uint32_t)FD_M;
#pragma unroll
    for (int j = 0; j < ND; j++) acc[i + j] += (uint64_t)m * (uint32_t)FD_P28[j];
    acc[i + 1] += (uint64_t)((int64_t)acc[i] >> 28);
  }
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < ND - 1; k++) {
    const int64_t v = (int64_t)acc[ND + k] + c;
    r[k] = (int32_t)(v & FD_M);
    c = v >> 28;
  }
  r[ND - 1] = (int32_t)((int64_t)acc[2 * ND - 1] + c);
}

// squaring: the 91 cross products once against a doubled digit
BGV_HD void fd_sqr_core(int32_t r[ND], const int32_t a[ND]) {
  uint64_t acc[2 * ND];
  int32_t d2[ND];
#pragma unroll
  for (int k = 0; k < 2 * ND; k++) acc[k] = 0;
#pragma unroll
  for (int k = 0; k < ND; k++) d2[k] = a[k] * 2;
#pragma unroll
  for (int i = 0; i < ND; i++) {
    acc[2 * i] += (uint64_t)((int64_t)a[i] * (int64_t)a[i]);
#pragma unroll
    for (int j = i + 1; j < ND; j++) acc[i + j] += (uint64_t)((int64_t)a[i] * (int64_t)d2[j]);
  }
#pragma unroll
  for (int i = 0; i < ND; i++) {
    const uint32_t m = ((uint32_t)acc[i] * FD_PINV) & (uint32_t)FD_M;
#pragma unroll
    for (int j = 0; j < ND; j++) acc[i + j] += (uint64_t)m * (uint32_t)FD_P28[j];
    acc[i + 1] += (uint64_t)((int64_t)acc[i] >> 28);
  }
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < ND - 1; k++) {
    const int64_t v = (int64_t)acc[ND + k] + c;
    r[k] = (int32_t)(v & FD_M);
    c = v >> 28;
  }
  r[ND - 1] = (int32_t)((int64_t)acc[2 * ND - 1] + c);
}

#if defined(__HIPCC__)
// register-ABI leaves (operands v0-v27, result v0-v13), one copy per unit
typedef int32_t fd_vec_t __attribute__((ext_vector_type(14)));
static __device__ __noinline__ fd_vec_t fd_mul_leaf(fd_vec_t a, fd_vec_t b) {
  int32_t x[ND], y[ND], z[ND];
#pragma unroll
  for (int k = 0; k < ND; k++) {
    x[k] = a[k];
    y[k] = b[k];
  }
  fd_mul_core(z, x, y);
  fd_vec_t v;
#pragma unroll
  for (int k = 0; k < ND; k++) v[k] = z[k];
  return v;
}
static __device__ __noinline__ fd_vec_t fd_sqr_leaf(fd_vec_t a) {
  int32_t x[ND], z[ND];
#pragma unroll
  for (int k = 0; k < ND; k++) x[k] = a[k];
  fd_sqr_core(z, x);
  fd_vec_t v;
#pragma unroll
  for (int k = 0; k < ND; k++) v[k] = z[k];
  return v;
}
#endif

BGV_HD void fd_mul(fd_t& r, const fd_t& a, const fd_t& b) {
#if !defined(__HIPCC__) && defined(BGV_FD_CHECK)
  fd_check_mul(a, b);
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  fd_vec_t va, vb;
#pragma unroll
  for (int k = 0; k < ND; k++) {
    va[k] = a.d[k];
    vb[k] = b.d[k];
  }
  const fd_vec_t vr = fd_mul_leaf(va, vb);
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = vr[k];
#else
  int32_t z[ND];
  fd_mul_core(z, a.d, b.d);
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = z[k];
#endif
}

BGV_HD void fd_sqr(fd_t& r, const fd_t& a) {
#if !defined(__HIPCC__) && defined(BGV_FD_CHECK)
  fd_check_mul(a, a);
  FD_ASSERT(fd_digit_max(a) < 1073741824.0, "squaring digit >= 2^30");
#endif
#if defined(__HIP_DEVICE_COMPILE__)
  fd_vec_t va;
#pragma unroll
  for (int k = 0; k < ND; k++) va[k] = a.d[k];
  const fd_vec_t vr = fd_sqr_leaf(va);
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = vr[k];
#else
  int32_t z[ND];
  fd_sqr_core(z, a.d);
#pragma unroll
  for (int k = 0; k < ND; k++) r.d[k] = z[k];
#endif
}

// ---- conversions to and from fp.h (canonical, R = 2^384) ---------------------
// digits of x 2^384 (x < p), then one product by 2^400: x 2^392
BGV_HD void fd_from_fp(fd_t& r, const fp_t& a) {
  fd_t t;
#pragma unroll
  for (int k = 0; k < ND; k++) {
    const int pos = 28 * k, w = pos >> 5, sh = pos & 31;
    const uint32_t lo = w < NL ? a.l[w] : 0u;
    const uint32_t hi = (w + 1) < NL ? a.l[w + 1] : 0u;
    const uint32_t v = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    t.d[k] = (int32_t)(v & (uint32_t)FD_M);
  }
  fd_mul(r, t, FD_C_IN);
}

// exact canonical digits of v in [0, p) for a product output v in (-p, 2p):
// carries propagated in order, then +p / -p by sign and comparison
BGV_HD void fd_canon(fd_t& r, const fd_t& a) {
  fd_t t;
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < ND - 1; k++) {
    const int64_t v = (int64_t)a.d[k] + c;
    t.d[k] = (int32_t)(v & FD_M);
    c = v >> 28;
  }
  t.d[ND - 1] = (int32_t)(a.d[ND - 1] + c);
  // negative: add p
  const int32_t neg = t.d[ND - 1] < 0;
  c = 0;
#pragma unroll
  for (int k = 0; k < ND; k++) {
    const int64_t v = (int64_t)t.d[k] + (neg ? FD_P28[k] : 0) + c;
    t.d[k] = k < ND - 1 ? (int32_t)(v & FD_M) : (int32_t)v;
    c = v >> 28;
  }
  // >= p: subtract p
  fd_t u;
  c = 0;
#pragma unroll
  for (int k = 0; k < ND; k++) {
    const int64_t v = (int64_t)t.d[k] - FD_P28[k] + c;
    u.d[k] = k < ND - 1 ? (int32_t)(v & FD_M) : (int32_t)v;
    c = v >> 28;
  }
  const bool ge = u.d[ND - 1] >= 0;
  fd_select(r, ge, u, t);
}

// x 2^392 -> x 2^384 (one product by 2^384), canonical, packed to 12 x u32
BGV_HD void fd_to_fp(fp_t& r, const fd_t& a) {
  fd_t t, c;
  fd_mul(t, a, FD_C_OUT);
  fd_canon(c, t);
#pragma unroll
  for (int m = 0; m < NL; m++) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < ND; k++) {
      const int rel = 28 * k - 32 * m;
      if (rel >= 32 || rel <= -28) continue;
      v |= rel >= 0 ? ((uint32_t)c.d[k] << rel) : ((uint32_t)c.d[k] >> (-rel));
    }
    r.l[m] = v;
  }
}

// v == 0 (mod p): fold to |v| < 0.6 p, exact canonical digits, compare
BGV_HD bool fd_is_zero(const fd_t& a) {
  fd_t t, c;
  fd_fold(t, a);
  fd_canon(c, t);
  int32_t acc = 0;
#pragma unroll
  for (int k = 0; k < ND; k++) acc |= c.d[k];
  return acc == 0;
}

// ---- Fp2 over fd ------------------------------------------------------------
BGV_HD void fd2_add(fd2_t& r, const fd2_t& a, const fd2_t& b) { fd_add(r.c0, a.c0, b.c0); fd_add(r.c1, a.c1, b.c1); }
BGV_HD void fd2_sub(fd2_t& r, const fd2_t& a, const fd2_t& b) { fd_sub(r.c0, a.c0, b.c0); fd_sub(r.c1, a.c1, b.c1); }
BGV_HD void fd2_neg(fd2_t& r, const fd2_t& a) { fd_neg(r.c0, a.c0); fd_neg(r.c1, a.c1); }
BGV_HD void fd2_dbl(fd2_t& r, const fd2_t& a) { fd_dbl(r.c0, a.c0); fd_dbl(r.c1, a.c1); }
template <int C> BGV_HD void fd2_mulc(fd2_t& r, const fd2_t& a) { fd_mulc<C>(r.c0, a.c0); fd_mulc<C>(r.c1, a.c1); }
BGV_HD void fd2_conj(fd2_t& r, const fd2_t& a) { r.c0 = a.c0; fd_neg(r.c1, a.c1); }
BGV_HD void fd2_norm(fd2_t& r, const fd2_t& a) { fd_norm(r.c0, a.c0); fd_norm(r.c1, a.c1); }
BGV_HD void fd2_fold(fd2_t& r, const fd2_t& a) { fd_fold(r.c0, a.c0); fd_fold(r.c1, a.c1); }
BGV_HD void fd2_select(fd2_t& r, bool c, const fd2_t& a, const fd2_t& b) {
  fd_select(r.c0, c, a.c0, b.c0);
  fd_select(r.c1, c, a.c1, b.c1);
}
// xi = 1 + i: (a0 - a1) + (a0 + a1) i
BGV_HD void fd2_mul_xi(fd2_t& r, const fd2_t& a) {
  fd_t t0, t1;
  fd_sub(t0, a.c0, a.c1);
  fd_add(t1, a.c0, a.c1);
  r.c0 = t0;
  r.c1 = t1;
}
BGV_HD void fd2_mul_fd(fd2_t& r, const fd2_t& a, const fd_t& b) { fd_mul(r.c0, a.c0, b); fd_mul(r.c1, a.c1, b); }
BGV_HD bool fd2_is_zero(const fd2_t& a) { return fd_is_zero(a.c0) && fd_is_zero(a.c1); }
BGV_HD void fd2_from_fp2(fd2_t& r, const fp2_t& a) { fd_from_fp(r.c0, a.c0); fd_from_fp(r.c1, a.c1); }
BGV_HD void fd2_to_fp2(fp2_t& r, const fd2_t& a) { fd_to_fp(r.c0, a.c0); fd_to_fp(r.c1, a.c1); }
BGV_HD fd2_t fd2_zero() { fd2_t r; fd_zero(r.c0); fd_zero(r.c1); return r; }
BGV_HD fd2_t fd2_one() { fd2_t r; r.c0 = FD_ONE; fd_zero(r.c1); return r; }

// schoolbook Fp2 product (4 Fp products, no operand sums: the value bound of
// each product is that of its inputs), one lane
BGV_HD void fd2_mul(fd2_t& r, const fd2_t& a, const fd2_t& b) {
  fd_t t0, t1, t2, t3;
  fd_mul(t0, a.c0, b.c0);
  fd_mul(t1, a.c1, b.c1);
  fd_mul(t2, a.c0, b.c1);
  fd_mul(t3, a.c1, b.c0);
  fd_sub(r.c0, t0, t1);
  fd_add(r.c1, t2, t3);
}

}  // namespace bgv
