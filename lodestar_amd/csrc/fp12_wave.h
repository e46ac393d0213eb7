// Wave-cooperative Fp12 arithmetic: one 64-lane workgroup works on ONE
// Fp12 value held in LDS, so a single final exponentiation (the batch
// check of maybeBatch.ts:18 / blst finalverify) runs at the latency of one
// Fp2 product per Fp12 multiplication instead of 54 sequential Fp products
// on one lane.
//
// Basis: Fp12 = Fp2[w] / (w^6 - xi); coefficient k (k = 0..5) of w^k sits
// at tower slot k=0 c0.c0, 1 c1.c0, 2 c0.c1, 3 c1.c1, 4 c0.c2, 5 c1.c2
// (fp12.h).  A product is the 6 x 6 schoolbook: lane l < 36 forms
// a_i * b_j (i = l / 6, j = l % 6), times xi when i + j >= 6; lanes 0..5
// then sum the six products landing on w^k.  Every function must be called
// by all 64 lanes of the workgroup (it contains __syncthreads()).
#pragma once
#include "fp12.h"

namespace bgv {

struct wfp12 {
  fp2_t c[6];
};

struct wscratch {
  fp2_t prod[36];
  wfp12 t[6];  // temporaries of the final exponentiation
};

__device__ __forceinline__ void w_from_tower(wfp12& r, const fp12_t& f) {
  r.c[0] = f.c0.c0; r.c[1] = f.c1.c0; r.c[2] = f.c0.c1;
  r.c[3] = f.c1.c1; r.c[4] = f.c0.c2; r.c[5] = f.c1.c2;
}

__device__ __forceinline__ void w_to_tower(fp12_t& f, const wfp12& r) {
  f.c0.c0 = r.c[0]; f.c1.c0 = r.c[1]; f.c0.c1 = r.c[2];
  f.c1.c1 = r.c[3]; f.c0.c2 = r.c[4]; f.c1.c2 = r.c[5];
}

// out = a * b (out may alias a or b)
__device__ void w_mul(wfp12* out, const wfp12* a, const wfp12* b, wscratch* s) {
  const uint32_t l = threadIdx.x;
  if (l < 36) {
    const uint32_t i = l / 6, j = l % 6;
    fp2_t t;
    fp2_mul(t, a->c[i], b->c[j]);
    if (i + j >= 6) fp2_mul_xi(t, t);
    s->prod[l] = t;
  }
  __syncthreads();
  if (l < 6) {
    fp2_t acc = s->prod[l];  // i = 0, j = l
#pragma unroll
    for (uint32_t i = 1; i < 6; i++) {
      const uint32_t j = (l + 6 - i) % 6;
      fp2_add(acc, acc, s->prod[i * 6 + j]);
    }
    out->c[l] = acc;
  }
  __syncthreads();
}

__device__ void w_copy(wfp12* out, const wfp12* a) {
  const uint32_t l = threadIdx.x;
  if (l < 6) out->c[l] = a->c[l];
  __syncthreads();
}

// conjugation over Fp6 (= inverse in the cyclotomic subgroup): negate odd w^k
__device__ void w_conj(wfp12* out, const wfp12* a) {
  const uint32_t l = threadIdx.x;
  if (l < 6) {
    fp2_t t = a->c[l];
    if (l & 1) fp2_neg(t, t);
    out->c[l] = t;
  }
  __syncthreads();
}

// Frobenius pi^k, k = 1..3 (fp12_frob)
__device__ void w_frob(wfp12* out, const wfp12* a, int k) {
  const uint32_t l = threadIdx.x;
  if (l < 6) {
    fp2_t t = a->c[l];
    if (k & 1) fp2_conj(t, t);
    if (l) fp2_mul(t, t, FROB_G[k - 1][l - 1]);
    out->c[l] = t;
  }
  __syncthreads();
}

// out = a^x (x < 0) for a in the cyclotomic subgroup
__device__ void w_pow_x(wfp12* out, const wfp12* a, wfp12* acc, wscratch* s) {
  w_copy(acc, a);
  for (int b = 62; b >= 0; b--) {
    w_mul(acc, acc, acc, s);
    if ((BLS_X_ABS >> b) & 1ull) w_mul(acc, acc, a, s);
  }
  w_conj(out, acc);
}

// Final exponentiation with the same addition chain as fp12_final_exp;
// returns (to every lane) whether the result is 1.
__device__ bool w_final_exp_is_one(const fp12_t& f_in, wscratch* s) {
  const uint32_t l = threadIdx.x;
  wfp12 *t0 = &s->t[0], *t1 = &s->t[1], *y0 = &s->t[2], *y1 = &s->t[3], *y2 = &s->t[4], *acc = &s->t[5];
  __shared__ wfp12 fin, y3;
  __shared__ uint32_t result;
  if (l == 0) {
    // the single Fp12 inversion of the easy part stays on one lane
    fp12_t inv;
    fp12_inv(inv, f_in);
    w_from_tower(*t0, inv);
    w_from_tower(fin, f_in);
  }
  __syncthreads();
  w_conj(t1, &fin);
  w_mul(t1, t1, t0, s);       // f^(p^6 - 1)
  w_frob(t0, t1, 2);
  w_mul(t1, t0, t1, s);       // m = f^((p^6-1)(p^2+1))
  w_pow_x(t0, t1, acc, s);
  w_conj(y0, t1);
  w_mul(y0, t0, y0, s);       // m^(x-1)
  w_pow_x(t0, y0, acc, s);
  w_conj(y1, y0);
  w_mul(y1, t0, y1, s);       // m^((x-1)^2)
  w_pow_x(t0, y1, acc, s);
  w_frob(y2, y1, 1);
  w_mul(y2, t0, y2, s);       // y1^(x + p)
  w_pow_x(t0, y2, acc, s);
  w_pow_x(t0, t0, acc, s);    // y2^(x^2)
  w_frob(&y3, y2, 2);
  w_mul(&y3, t0, &y3, s);
  w_conj(t0, y2);
  w_mul(&y3, &y3, t0, s);     // y2^(x^2 + p^2 - 1)
  w_mul(t0, t1, t1, s);
  w_mul(t0, t0, t1, s);       // m^3
  w_mul(&y3, &y3, t0, s);
  if (l == 0) {
    fp12_t r;
    w_to_tower(r, y3);
    result = fp12_is_one(r) ? 1u : 0u;
  }
  __syncthreads();
  return result != 0;
}

}  // namespace bgv
