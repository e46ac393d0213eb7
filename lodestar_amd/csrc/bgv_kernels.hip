// HIP kernels of the gfx950 BLS12-381 batch verifier.
//
// One device batch flows through these stages on the context's stream
// (host orchestration: bgv_api.hip).  Every stage is one lane per signature
// set (or per job): the per-set work is a long chain of dependent 384-bit
// Montgomery products on the integer VALU, so the lane is the natural unit
// and sets are independent.
//
//   k_raw_pks     raw (non-table) pubkeys  -> Montgomery affine G1
//   k_sig         Signature.fromBytes(sig, affine, validate=true)
//                 (maybeBatch.ts:23,36): length check, ZCash decode,
//                 on-curve, G2 subgroup check (psi(P) == [x]P)
//   k_hash        hash_to_G2(signingRoot, POP DST) -> affine H(m)
//   k_pk          PublicKey.aggregate (chain/bls/utils.ts:11) as a gather
//                 from the HBM index2pubkey table + [r_i] PK_i (mul_n_aggregate)
//   k_sig_scale   [r_i] sigma_i
//   k_miller      f_i = MillerLoop([r_i] PK_i, H(m_i))
//   k_job         per job: f_j = prod f_i * MillerLoop(-G1, sum [r_i] sigma_i),
//                 first parse error of the job (set order)
//   (bgv_tail.hip) per-job and whole-batch Fp12 product trees, ONE final
//                 exponentiation for the batch, per-job final exponentiation
//                 only if the batch check failed (the worker's per-job retry,
//                 multithread/worker.ts:74-85)
// Code generation of this translation unit (measured on MI355X, r01):
//  * every Fp product is a call to one non-inlined leaf with its operands in
//    VGPRs (fp.h BGV_FPMUL_CALL) and the Fp2 and Fp6 layers are inlined, so
//    their temporaries live in registers instead of on the scratch stack
//    (Fp6 inlining: k_miller 33.5 -> 30.5 ms);
//  * the Miller kernel runs at 1 wave/SIMD: its 512-register budget takes
//    the spills in AGPRs (k_miller 37.9 -> 33.1 ms at C4).
// The Fp12 product trees and final exponentiations prefer the inlined
// product and live in bgv_tail.hip.
#ifndef BGV_FPMUL_CALL
#define BGV_FPMUL_CALL 1
#endif
#ifndef BGV_FP2_INLINE
#define BGV_FP2_INLINE 1
#endif
#ifndef BGV_FP6_INLINE
#define BGV_FP6_INLINE 1
#endif
#ifndef BGV_POINT_INLINE
#define BGV_POINT_INLINE 1  // jac_dbl / jac_add / jac_add_aff: 2049k -> 2155k sets/s
#endif
#ifndef BGV_MILLER_WAVES
#define BGV_MILLER_WAVES 1
#endif
#ifndef BGV_MILLER_LDS_F
#define BGV_MILLER_LDS_F 1
#endif
// The Fp2 leaf (fp2.h BGV_FP2_LEAF) stays off in this unit: its 48-dword
// argument frame pushes k_hash over the 256-register line of two waves per
// SIMD (k_hash 16.0 -> 17.7 ms alone; profiles/r06i_fp2_leaf/).  The Miller
// and latency units take it.  BGV_KERNELS_FP2_LEAF=1 builds the A/B variant.
#ifndef BGV_KERNELS_FP2_LEAF
#define BGV_KERNELS_FP2_LEAF 0
#endif
#ifndef BGV_FP2_LEAF
#define BGV_FP2_LEAF BGV_KERNELS_FP2_LEAF
#endif
#include "bgv_internal.h"
#include "miller_coop.h"

namespace bgv {

// Occupancy of the per-set kernels: minimum waves per SIMD requested from the
// register allocator (1 = up to 512 VGPR+AGPR per lane).  Tuned on MI355X.
#ifndef BGV_WAVES
#define BGV_WAVES 2
#endif
#define BGV_BULK __launch_bounds__(64, BGV_WAVES)
#ifndef BGV_HASH_WAVES
#define BGV_HASH_WAVES BGV_WAVES
#endif
#ifndef BGV_SIG_WAVES
#define BGV_SIG_WAVES BGV_WAVES
#endif
#ifndef BGV_SCALE_WAVES
#define BGV_SCALE_WAVES BGV_WAVES
#endif
#ifndef BGV_PK_WAVES
#define BGV_PK_WAVES BGV_WAVES
#endif
#ifndef BGV_MILLER_WAVES
#define BGV_MILLER_WAVES BGV_WAVES
#endif

__device__ __forceinline__ uint32_t gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }

// ---------------------------------------------------------------- helpers
// ------------------------------------------------------------ k_raw_pks
// uncompressed 96 B big-endian, trusted (multithread/worker.ts:108-114:
// PublicKey.fromBytes(.., affine) without validation); infinity -> (0, 0)
__global__ void BGV_BULK k_raw_pks(const uint8_t* raw, g1a* out, uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  g1a p;
  if (!g1_from_uncompressed_trusted(p, raw + 96u * i)) { fp_set_zero(p.x); fp_set_zero(p.y); }
  out[i] = p;
}

// compressed 48 B table load (syncPubkeys path: PublicKey.fromBytes(pk,
// jacobian) without validation, pubkeyCache.ts:75): decode + on-curve, the
// infinity key is stored as (0, 0) and adds nothing to an aggregate; codes[i]
// is the blst code of a key that does not decode (the host rejects the call)
__global__ void BGV_BULK k_table_from_compressed(const uint8_t* in48, g1a* out, uint32_t n, int32_t* codes) {
  const uint32_t i = gtid();
  if (i >= n) return;
  g1a p;
  bool inf;
  const int32_t c = g1_decompress(p, inf, in48 + 48u * i);
  if (c != C_OK || inf) { fp_set_zero(p.x); fp_set_zero(p.y); }
  out[i] = p;
  codes[i] = c;
}

// 96 B uncompressed (x || y big-endian): blst deserialization checks the
// flags, x, y < p and the curve equation (no subgroup check)
__global__ void BGV_BULK k_table_from_uncompressed(const uint8_t* in96, g1a* out, uint32_t n, int32_t* codes) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const uint8_t* b = in96 + 96u * i;
  g1a p;
  fp_set_zero(p.x);
  fp_set_zero(p.y);
  int32_t c = C_OK;
  if (b[0] & 0x80) {
    c = C_BAD_ENCODING;  // compressed flag on a 96-byte key
  } else if (b[0] & 0x40) {  // infinity: every other bit zero
    uint32_t acc = b[0] & 0x3f;
    for (int k = 1; k < 96; k++) acc |= b[k];
    if (acc) c = C_BAD_ENCODING;
  } else {
    fp_t x, y;
    fp_from_be48(x, b);
    fp_from_be48(y, b + 48);
    if ((b[0] & 0x20) || !fp_plain_lt_p(x) || !fp_plain_lt_p(y)) {
      c = C_BAD_ENCODING;
    } else {
      fp_to_mont(p.x, x);
      fp_to_mont(p.y, y);
      fp_t y2, x3;
      fp_sqr(y2, p.y);
      fp_sqr(x3, p.x);
      fp_mul(x3, x3, p.x);
      fp_add(x3, x3, B1_MONT);
      if (!fp_eq(y2, x3)) {
        c = C_POINT_NOT_ON_CURVE;
        fp_set_zero(p.x);
        fp_set_zero(p.y);
      }
    }
  }
  out[i] = p;
  codes[i] = c;
}

__global__ void BGV_BULK k_table_export(const g1a* tab, uint8_t* out96, uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const g1a p = tab[i];
  uint8_t* o = out96 + 96u * i;
  if (g1a_is_zero(p)) {
    for (int k = 0; k < 96; k++) o[k] = 0;
    o[0] = 0x40;
    return;
  }
  fp_t t;
  fp_from_mont(t, p.x);
  fp_to_be48(o, t);
  fp_from_mont(t, p.y);
  fp_to_be48(o + 48, t);
}

// plain big-endian export of affine points (bgv_debug_stages): x then y,
// Fp2 coordinates as c0 || c1; the identity (0, 0) stays all-zero
__global__ void BGV_BULK k_export_g1a(const g1a* in, uint8_t* out96, uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const g1a p = in[i];
  fp_t t;
  fp_from_mont(t, p.x);
  fp_to_be48(out96 + 96u * i, t);
  fp_from_mont(t, p.y);
  fp_to_be48(out96 + 96u * i + 48, t);
}

__global__ void BGV_BULK k_export_g2a(const g2a* in, uint8_t* out192, uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const g2a p = in[i];
  const fp_t* c[4] = {&p.x.c0, &p.x.c1, &p.y.c0, &p.y.c1};
  for (int k = 0; k < 4; k++) {
    fp_t t;
    fp_from_mont(t, *c[k]);
    fp_to_be48(out192 + 192u * i + 48 * k, t);
  }
}

// ------------------------------------------------------------------ k_sig
__global__ void __launch_bounds__(64, BGV_SIG_WAVES) k_sig(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const uint32_t len = b.sig_len[i];
  const uint8_t* s = b.sigs + 192u * i;
  g2a a;
  bool inf = false;
  int32_t code;
  if (len == 96u) code = g2_decompress(a, inf, s);
  else if (len == 192u) code = g2_deserialize(a, inf, s);
  else code = C_INVALID_SIZE;
  // partial deferral (dev_batch.defer_from): sets from defer_from on are
  // checked later by launch_sig_check (wave-uniform: a multiple of 64)
  if (code == C_OK && !inf && !(b.defer_grp && i >= b.defer_from)) {
    g2j j;
    jac_from_aff(j, a);
    if (!g2_in_subgroup(j)) code = C_POINT_NOT_IN_GROUP;
  }
  if (code != C_OK || inf) { a.x = fp2_zero(); a.y = fp2_zero(); }
  w.sig_aff[i] = a;
  w.sig_inf[i] = inf ? 1u : 0u;
  w.sig_code[i] = code;
}

// Latency mode (dev_batch.split, small batches): the decode runs alone, then
// one launch runs the subgroup check and [r_i] sigma_i side by side (blocks
// [0, nb) check, blocks [nb, 2 nb) scale: uniform per wave), so the
// signature path's chain is decode + max(check, scale) instead of
// decode + check + scale.  k_sig_fix folds the check into the codes.
__global__ void __launch_bounds__(64, BGV_SIG_WAVES) k_sig_dec(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const uint32_t len = b.sig_len[i];
  const uint8_t* s = b.sigs + 192u * i;
  g2a a;
  bool inf = false;
  int32_t code;
  if (len == 96u) code = g2_decompress(a, inf, s);
  else if (len == 192u) code = g2_deserialize(a, inf, s);
  else code = C_INVALID_SIZE;
  if (code != C_OK || inf) { a.x = fp2_zero(); a.y = fp2_zero(); }
  w.sig_aff[i] = a;
  w.sig_inf[i] = inf ? 1u : 0u;
  w.sig_code[i] = code;
}

__global__ void __launch_bounds__(64, BGV_SIG_WAVES) k_sig_split(dev_batch b, dev_work w) {
  const uint32_t nb = (b.n_sets + 63u) / 64u;
  const bool check = blockIdx.x < nb;
  // deferred checks (launch_sig_check) start at defer_from
  const uint32_t i = (check ? blockIdx.x : blockIdx.x - nb) * 64u + threadIdx.x + (check && b.defer_grp ? b.defer_from : 0u);
  if (i >= b.n_sets) return;
  const bool live = w.sig_code[i] == C_OK && !w.sig_inf[i];  // decode outcome (k_sig_dec)
  if (check) {
    uint32_t ok = 1u;
    if (live) {
      g2j j;
      jac_from_aff(j, w.sig_aff[i]);
      ok = g2_in_subgroup(j) ? 1u : 0u;
    }
    w.sig_grp[i] = ok;
  } else {
    g2j r;
    if (!live) {
      jac_set_inf(r);
    } else {
      g2j s;
      jac_from_aff(s, w.sig_aff[i]);
      jac_mul_u64_w4(r, s, b.scalars[i]);
    }
    w.rsig[i] = r;
  }
}

__global__ void BGV_BULK k_sig_fix(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets || (b.defer_grp && i < b.defer_from)) return;  // checked in ST_SIG
  if (w.sig_code[i] == C_OK && !w.sig_grp[i]) {
    w.sig_code[i] = C_POINT_NOT_IN_GROUP;
    g2a z;
    z.x = fp2_zero();
    z.y = fp2_zero();
    w.sig_aff[i] = z;
  }
}

// Deferred subgroup check (bulk mode, dev_batch.defer_grp).  The signature
// stage only decodes, so the MSM starts ~60% sooner and phase 1 of the step
// (hash, pubkeys, decode) carries ~1,200 fewer Fp products per set; the
// checks run beside the set-pair Miller loops on the SIMDs it leaves free.
// Their verdicts reach the codes before anything reads them: k_sig_fix marks
// the failing signatures, k_job_recode re-derives every job's first failing
// code (signatures first, then pubkeys, maybeBatch.ts:20-24) and gives a job
// that only now fails the identity S_job and (-G1, S_job) value, exactly what
// a job rejected at decode time has (k_msm_job / k_miller_coop), so the fold
// leaves it out of the batch product.
__global__ void BGV_BULK k_job_recode(dev_batch b, dev_work w) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  // every job: a subgroup failure of an earlier set takes precedence over a
  // decode failure of a later one (first failing code in set order)
  const int32_t was = w.job_code[j];
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  int32_t code = C_OK;
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.sig_code[i];
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.pk_code[i];
  if (end == beg) code = C_EMPTY_JOB;
  if (code == was) return;
  w.job_code[j] = code;
  if (was != C_OK) return;  // rejected at decode time: S_job and its pair are already the identity
  g2a z;
  z.x = fp2_zero();
  z.y = fp2_zero();
  w.s_aff[j] = z;
  w.s_inf[j] = 1u;
  fp12_t one;
  fp12_one(one);
  w.f_set[b.n_sets + j] = one;
}

// The cooperative G2 kernels of the latency mode (k_sig_split_coop,
// k_hash_clear_coop) live in bgv_latency.hip: they run at 1 wave/SIMD, and
// sharing this unit's non-inlined curve helpers with them raised k_sig to
// 321 VGPRs (1 wave/SIMD; C4 sig decode 6 -> 21 ms).
#ifndef BGV_COOP_G2
#define BGV_COOP_G2 1
#endif
#ifndef BGV_MSM_JOB_COOP
#define BGV_MSM_JOB_COOP 1
#endif
#ifndef BGV_PK_COOP
#define BGV_PK_COOP 1
#endif
#ifndef PK_COOP_MAX
#define PK_COOP_MAX 9000u  // 3,136 sets: 7.20 -> 6.68 ms; at 12,544 its waves slow the clearing (9.7 -> 10.3 ms)
#endif
#ifndef BGV_MSM_JOB_COOP_BULK
#define BGV_MSM_JOB_COOP_BULK 0
#endif

// latency mode: lane t maps u_(t & 1) of message t >> 1; then one lane per
// message adds the two points and clears the cofactor
__global__ void __launch_bounds__(64, BGV_HASH_WAVES) k_hash_map(dev_batch b, dev_work w) {
  const uint32_t t = gtid();
  if (t >= 2u * b.n_sets) return;
  const uint32_t i = t >> 1;
  uint8_t m[32];
#pragma unroll
  for (int k = 0; k < 32; k++) m[k] = b.msgs[32u * i + k];
  g2j q;
  hash_to_g2_map(q, m, t & 1u);
  w.q_part[t] = q;
}

__global__ void __launch_bounds__(64, BGV_HASH_WAVES) k_hash_clear(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  g2j h;
  hash_to_g2_finish(h, w.q_part[2u * i], w.q_part[2u * i + 1u]);
  g2a ha;
  jac_to_aff(ha, h);
  w.h_aff[i] = ha;
}

// ----------------------------------------------------------------- k_hash
__global__ void __launch_bounds__(64, BGV_HASH_WAVES) k_hash(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  uint8_t m[32];
#pragma unroll
  for (int k = 0; k < 32; k++) m[k] = b.msgs[32u * i + k];
  g2j h;
  hash_to_g2(h, m);
  g2a ha;
  jac_to_aff(ha, h);  // H(m) is never the identity for a 32-byte root (prob. 2^-255)
  w.h_aff[i] = ha;
}

// ------------------------------------------------------------------- k_pk
// PublicKey.aggregate as a balanced gather: every set's index list is cut
// into chunks of PK_CHUNK keys (a 512-key sync-committee set is 16 chunks,
// a 128-key attestation 4, a single 1) so lanes of one wave do equal work;
// chunk offsets come from a device scan.  Then one lane per set folds its
// chunk sums, applies the batch scalar r_i and converts to affine.

// Offsets that run backwards (an on-device batch that breaks the contract;
// host batches are checked by the library) give the set no chunks, and the
// chunk scan is clipped at chunk_bound below: no access leaves the buffers.
__global__ void BGV_BULK k_chunk_count(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const uint32_t lo = b.pk_off[i], hi = b.pk_off[i + 1];
  const uint32_t k = hi > lo ? hi - lo : 0u;
  w.chunk_off[i] = (k + PK_CHUNK - 1) / PK_CHUNK;
}

// exclusive scan of a[0..n) in place, total at a[n]; one workgroup walking
// 1024-element tiles with coalesced loads: wave scan by shuffles, the 16 wave
// totals scanned by wave 0, a running carry across tiles
__global__ void __launch_bounds__(1024) k_scan(uint32_t* a, uint32_t n) {
  __shared__ uint32_t wsum[16];
  const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n; base += 1024u) {
    const uint32_t i = base + t;
    const uint32_t v = i < n ? a[i] : 0u;
    uint32_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (wid == 0) {
      uint32_t s = lane < 16 ? wsum[lane] : 0u;
#pragma unroll
      for (uint32_t d = 1; d < 16; d <<= 1) {
        const uint32_t y = __shfl_up(s, d, 64);
        if (lane >= d) s += y;
      }
      if (lane < 16) wsum[lane] = s;
    }
    __syncthreads();
    if (i < n) a[i] = carry + (wid ? wsum[wid - 1] : 0u) + x - v;
    carry += wsum[15];
    __syncthreads();  // wsum is rewritten by the next tile
  }
  if (t == 0) a[n] = carry;
}

__global__ void BGV_BULK k_chunk_set(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const uint32_t end = min(w.chunk_off[i + 1], b.chunk_bound);
  for (uint32_t c = w.chunk_off[i]; c < end; c++) w.chunk_set[c] = i;
}

// k_pk_chunk (the gather) lives in bgv_gather.hip: it runs with the product
// inlined, so the next row's load stays in flight across the additions

__global__ void __launch_bounds__(64, BGV_PK_WAVES) k_pk(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  g1j acc;
  jac_set_inf(acc);
  const uint32_t c0 = w.chunk_off[i], c1 = w.chunk_off[i + 1];
  bool range_err = c1 > b.chunk_bound || b.pk_off[i + 1] < b.pk_off[i];
  for (uint32_t c = c0; c < c1 && !range_err; c++) {
    const g1j p = w.pk_part[c];
    if (!jac_is_inf(p) && fp_is_zero(p.x)) range_err = true;
    jac_add(acc, acc, p);
  }
  int32_t code = C_OK;
  if (range_err) code = C_INDEX_RANGE;
  else if (jac_is_inf(acc)) code = C_PK_IS_INFINITY;
  g1a out;
  if (w.pk_agg) {  // bgv_debug_stages: the aggregate before scaling
    if (code != C_OK || !jac_to_aff(out, acc)) { fp_set_zero(out.x); fp_set_zero(out.y); }
    w.pk_agg[i] = out;
  }
  if (code == C_OK) {
    g1j rp;
    jac_mul_u64_w4(rp, acc, b.scalars[i]);
    jac_to_aff(out, rp);
  } else {
    fp_set_zero(out.x);
    fp_set_zero(out.y);
  }
  w.rpk_aff[i] = out;
  w.pk_code[i] = code;
}

// ------------------------------------------------------------ k_sig_scale
__global__ void __launch_bounds__(64, BGV_SCALE_WAVES) k_sig_scale(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  g2j r;
  if (w.sig_code[i] != C_OK || w.sig_inf[i]) {
    jac_set_inf(r);  // infinity signature: blst skips it (adds the identity)
  } else {
    g2j s;
    jac_from_aff(s, w.sig_aff[i]);
    jac_mul_u64_w4(r, s, b.scalars[i]);
  }
  w.rsig[i] = r;
}

// ------------------------------------------- per-job bucket MSM (msm mode)
// S_job = sum_i r_i sigma_i over the job's sets with the 64-bit scalars cut
// into 16 windows of 4 bits (Pippenger): bucket d of window w holds the sum
// of the sigma_i whose digit w is d; S_w = sum_d d B_d by running sums;
// S_job = sum_w 16^w S_w by Horner.  Per 98-set job: 16 x 98 mixed additions
// + 16 x 30 additions + 60 doublings + 15 additions (~790 Fp-mul per set
// against 2,140 for a per-set 4-bit window multiplication).  Invalid and
// identity signatures add nothing: a job with a bad signature is rejected by
// its code and never reaches the pairing.

// msm = 2 (bulk batches): lane = (job, window); the 15 buckets live in HBM/L2, `mask` marks the
// occupied ones (an unoccupied bucket is the identity: no initialisation)
__global__ void BGV_BULK k_msm_bucket(dev_batch b, dev_work w) {
  const uint32_t t = gtid();
  if (t >= b.n_jobs * 16u) return;
  const uint32_t j = t >> 4, win = t & 15u;
  g2j* bk = w.msm_bucket + (size_t)t * 15u;
  uint32_t mask = 0;
  for (uint32_t i = b.job_off[j]; i < b.job_off[j + 1]; i++) {
    if (w.sig_code[i] != C_OK || w.sig_inf[i]) continue;
    const uint32_t d = (uint32_t)(b.scalars[i] >> (4u * win)) & 15u;
    if (d == 0) continue;
    const g2a s = w.sig_aff[i];
    g2j acc;
    if ((mask >> d) & 1u) {
      acc = bk[d - 1];
      jac_add_aff(acc, acc, s);
    } else {
      jac_from_aff(acc, s);
      mask |= 1u << d;
    }
    bk[d - 1] = acc;
  }
  w.msm_mask[t] = mask;
}

// lane = (job, window): S_w = sum_d d B_d = sum_{d'} (sum_{d >= d'} B_d)
__global__ void BGV_BULK k_msm_window(dev_batch b, dev_work w) {
  const uint32_t t = gtid();
  if (t >= b.n_jobs * 16u) return;
  const g2j* bk = w.msm_bucket + (size_t)t * 15u;
  const uint32_t mask = w.msm_mask[t];
  g2j run, tot;
  jac_set_inf(run);
  jac_set_inf(tot);
  for (uint32_t d = 15; d >= 1; d--) {
    if ((mask >> d) & 1u) {
      const g2j v = bk[d - 1];
      jac_add(run, run, v);
    }
    jac_add(tot, tot, run);
  }
  w.msm_win[t] = tot;
}

// msm = 4 (mid-size batches, latency mode): lane = (job, window w, digit d),
// 256 lanes per job (four windows per wave):
//   1. bucket d of window w: the mixed sum of the job's signatures whose
//      digit w is d, in registers (each lane walks the job's scalars to its
//      next match; the wave runs as many additions as its fullest bucket);
//   2. d B_d by MSB-first double-and-add (<= 3 doublings and additions);
//   3. S_w = sum_d d B_d by a tree over the window's 16 lanes (cross-lane
//      shuffles inside the wave, 4 levels); lane d = 0 writes S_w.
// No bucket leaves the registers; the chain is ~max-bucket mixed additions +
// 6 + 4 point operations (against the job's span + 30 of a (job, window)
// lane walking all its sets and then its running sums).  Bulk batches keep
// that form (msm = 2): a wave here runs its fullest bucket's additions, ~2x
// the mean, which at C4 costs phase 1 ~1.2 ms (same-box A/B, r03).
__device__ __forceinline__ void shfl_down16(g2j& r, const g2j& v, uint32_t st) {
  const uint32_t* src = (const uint32_t*)&v;
  uint32_t* dst = (uint32_t*)&r;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(g2j) / 4); k++) dst[k] = (uint32_t)__shfl_down((int)src[k], st, 16);
}

__global__ void BGV_BULK k_msm_digit(dev_batch b, dev_work w) {
  const uint32_t t = gtid();
  const uint32_t j = t >> 8, win = (t >> 4) & 15u, d = t & 15u;
  if (j >= b.n_jobs) return;  // whole waves: 256 lanes per job
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  g2j acc;
  jac_set_inf(acc);
  bool first = true;
  uint32_t i = beg;
  for (;;) {
    // this lane's next set whose digit in window `win` is d (digit 0 adds nothing)
    while (i < end) {
      const bool live = w.sig_code[i] == C_OK && !w.sig_inf[i];
      const uint32_t dig = (uint32_t)(b.scalars[i] >> (4u * win)) & 15u;
      if (live && d != 0 && dig == d) break;
      i++;
    }
    if (!__any(i < end)) break;
    if (i < end) {
      const g2a s = w.sig_aff[i];
      if (first) jac_from_aff(acc, s);
      else jac_add_aff(acc, acc, s);
      first = false;
      i++;
    }
  }
  // d B_d
  const g2j base = acc;
  for (int bit = 2; bit >= 0; bit--) {
    if (d >> (bit + 1)) {
      jac_dbl(acc, acc);
      if ((d >> bit) & 1u) jac_add(acc, acc, base);
    }
  }
  // S_w: lanes [st, 2 st) of the window hand their sums to lanes [0, st)
  for (uint32_t st = 8; st >= 1; st >>= 1) {
    g2j o;
    shfl_down16(o, acc, st);
    if (d < st) jac_add(acc, acc, o);
  }
  if (d == 0) w.msm_win[16u * j + win] = acc;
}

// per job: S_job = sum_w 16^w S_w, codes as k_job_s.  Lane (job, window w)
// doubles its window sum 4 w times, then a tree over the job's 16 lanes
// (cross-lane shuffles): 60 doublings + 4 additions on the chain instead of a
// one-lane Horner's 60 doublings + 15 additions
__global__ void BGV_BULK k_msm_job(dev_batch b, dev_work w) {
  const uint32_t t = gtid();
  const uint32_t j = t >> 4, win = t & 15u;
  if (j >= b.n_jobs) return;  // whole 16-lane groups (n_jobs * 16 lanes)
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  int32_t code = C_OK;
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.sig_code[i];
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.pk_code[i];
  if (end == beg) code = C_EMPTY_JOB;
  g2j s;
  jac_set_inf(s);
  if (code == C_OK) {
    s = w.msm_win[16u * j + win];
    for (uint32_t k = 0; k < 4u * win; k++) jac_dbl(s, s);
  }
  for (uint32_t st = 8; st >= 1; st >>= 1) {
    g2j o;
    shfl_down16(o, s, st);
    if (win < st) jac_add(s, s, o);
  }
  if (win != 0) return;
  g2a sa;
  sa.x = fp2_zero();
  sa.y = fp2_zero();
  uint32_t inf = 1;
  if (code == C_OK) inf = jac_to_aff(sa, s) ? 0u : 1u;
  w.s_aff[j] = sa;
  w.s_inf[j] = inf;
  w.job_code[j] = code;
}

// ------------------------------------------ fused per-job MSM (msm mode)
// One 256-lane workgroup per job computes S_job = sum_i r_i sigma_i with no
// bucket in HBM: lane (w, d) = (tid >> 4, tid & 15) owns bucket d of window
// w (4-bit windows of the 64-bit scalars).
//   1. counting sort, in LDS, of the job's sets by their digit in every
//      window (order[w][...] = set offsets grouped by digit);
//   2. lane (w, d) adds its sets' sigma (mixed additions, bucket in VGPRs):
//      ~span/16 additions per lane, the wave's lanes busy together;
//   3. B <- d B by double-and-add (d <= 15), then a tree over the 16 digits
//      of each window in LDS: S_w = sum_d d B_d;
//   4. lane (w, 0): T_w = 2^(4w) S_w (4w doublings), then a tree over the
//      windows: S_job = sum_w T_w; lane 0 converts to affine and writes the
//      job code (first failing set code, signatures before pubkeys).
// The dependent chain is ~max-bucket additions + 6 + 4 + 60 doublings + 4
// additions + one inversion, against span + 30 + 75 sequential operations of
// the (job, window)-lane form; 4 waves per job (4,096 at C4).  Invalid and
// identity signatures add nothing (their job is rejected by its code).
// S_job's affine value does not depend on the order of the additions.
constexpr uint32_t MSM_LANES = 256;
__global__ void __launch_bounds__(MSM_LANES, 1) k_msm_fused(dev_batch b, dev_work w, uint32_t chunk) {
  __shared__ g2j pts[128];                   // tree exchange (8 slots per window)
  extern __shared__ g2a sg[];                // the chunk's decoded signatures (dynamic: chunk x 192 B)
  __shared__ uint8_t order[16][256];         // set offsets by digit, per window
  __shared__ uint32_t cnt[16][16], start[16][17];
  const uint32_t j = blockIdx.x, tid = threadIdx.x, win = tid >> 4, dig = tid & 15u;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  g2j acc;
  jac_set_inf(acc);
  bool first = true;
  // jobs are sorted and summed `chunk` (<= 256) sets at a time (block-sized jobs: once)
  for (uint32_t c0 = beg; c0 < end; c0 += chunk) {
    const uint32_t n = min(end - c0, chunk);
    cnt[win][dig] = 0u;
    __syncthreads();
    // 1. digit histogram of every window (lane t takes set t)
    const bool live = tid < n && w.sig_code[c0 + tid] == C_OK && !w.sig_inf[c0 + tid];
    const uint64_t r = tid < n ? b.scalars[c0 + tid] : 0ull;
    // staged in LDS: the bucket additions below then wait on LDS, not HBM
    // (every product call begins with s_waitcnt on all outstanding loads)
    if (live) sg[tid] = w.sig_aff[c0 + tid];
    if (live)
      for (uint32_t ww = 0; ww < 16; ww++) atomicAdd(&cnt[ww][(uint32_t)(r >> (4u * ww)) & 15u], 1u);
    __syncthreads();
    if (dig == 0) {
      uint32_t a = 0;
      for (uint32_t d = 0; d < 16; d++) { start[win][d] = a; a += cnt[win][d]; }
      start[win][16] = a;
    }
    __syncthreads();
    cnt[win][dig] = 0u;
    __syncthreads();
    if (live)
      for (uint32_t ww = 0; ww < 16; ww++) {
        const uint32_t d = (uint32_t)(r >> (4u * ww)) & 15u;
        order[ww][start[ww][d] + atomicAdd(&cnt[ww][d], 1u)] = (uint8_t)tid;
      }
    __syncthreads();
    // 2. bucket (win, dig): its sets' signatures (digit 0 contributes nothing)
    if (dig != 0) {
      const uint32_t k0 = start[win][dig], k1 = start[win][dig + 1];
      for (uint32_t k = k0; k < k1; k++) {
        const g2a s = sg[order[win][k]];
        if (first) jac_from_aff(acc, s);
        else jac_add_aff(acc, acc, s);
        first = false;
      }
    }
    __syncthreads();  // order / start are rewritten by the next chunk
  }
  // 3. d B_d (MSB-first double-and-add), then the tree over the digits
  if (dig > 1 && !jac_is_inf(acc)) {
    const g2j base = acc;
    const int top = 31 - __clz((int)dig);
    for (int bit = top - 1; bit >= 0; bit--) {
      jac_dbl(acc, acc);
      if ((dig >> bit) & 1u) jac_add(acc, acc, base);
    }
  }
  // level st: digits [st, 2 st) hand their sums to digits [0, st)
  for (uint32_t st = 8; st >= 1; st >>= 1) {
    if (dig >= st && dig < 2u * st) pts[8u * win + dig - st] = acc;
    __syncthreads();
    if (dig < st) {
      g2j o = pts[8u * win + dig];
      jac_add(acc, acc, o);
    }
    __syncthreads();
  }
  // 4. T_w = 2^(4 w) S_w, then the tree over the windows
  if (dig == 0)
    for (uint32_t k = 0; k < 4u * win; k++) jac_dbl(acc, acc);
  for (uint32_t st = 8; st >= 1; st >>= 1) {
    if (dig == 0 && win >= st && win < 2u * st) pts[win - st] = acc;
    __syncthreads();
    if (dig == 0 && win < st) {
      g2j o = pts[win];
      jac_add(acc, acc, o);
    }
    __syncthreads();
  }
  if (tid == 0) {
    g2a sa;
    if (!jac_to_aff(sa, acc)) { sa.x = fp2_zero(); sa.y = fp2_zero(); }
    w.s_aff[j] = sa;
    w.s_inf[j] = jac_is_inf(acc) ? 1u : 0u;
  }
}

// per job, after the pubkeys (ST_S_TREE, k_msm_fused mode): the job code
// (first failing set, signatures before pubkeys, maybeBatch.ts:20-24); a
// rejected job's S_job becomes the identity, so its (-G1, S_job) pair is 1
__global__ void BGV_BULK k_job_code(dev_batch b, dev_work w) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  int32_t code = C_OK;
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.sig_code[i];
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.pk_code[i];
  if (end == beg) code = C_EMPTY_JOB;
  w.job_code[j] = code;
  if (code != C_OK) {
    g2a z;
    z.x = fp2_zero();
    z.y = fp2_zero();
    w.s_aff[j] = z;
    w.s_inf[j] = 1u;
  }
}

// ------------------------------------------------------ per-job S tree
// Sum of [r_i] sigma_i per job as a segmented pairwise tree: level `s`
// folds element i + s into i for every i at an even multiple of s inside
// its job.  log2(job size) launches replace a serial per-job loop (the
// first levels run on n/2 lanes, so the latency cost is one G2 add per level).
__global__ void BGV_BULK k_set_job(dev_batch b, dev_work w) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  for (uint32_t i = b.job_off[j]; i < b.job_off[j + 1]; i++) w.set_job[i] = j;
}

constexpr uint32_t S_COOP_MAX = 16384;  // ST_S_TREE: k_s_level_coop below, k_s_level above
__global__ void BGV_BULK k_s_level(dev_batch b, dev_work w, uint32_t s) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const uint32_t j = w.set_job[i];
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  if (((i - beg) % (2 * s)) != 0 || i + s >= end) return;
  g2j a = w.rsig[i];
  const g2j c = w.rsig[i + s];
  jac_add(a, a, c);
  w.rsig[i] = a;
}

// per job: first parse error (set order), S_job -> affine as the job's
// extra Miller pair (-G1, S_job) at pair index n_sets + j
__global__ void BGV_BULK k_job_s(dev_batch b, dev_work w, uint32_t span) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  const uint32_t beg = b.job_off[j], end = b.job_off[j + 1];
  // reference order: every signature of the job is parsed/validated first
  // (maybeBatch.ts:20-24 sets.map(fromBytes)), then blst reaches the pubkeys
  int32_t code = C_OK;
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.sig_code[i];
  for (uint32_t i = beg; i < end && code == C_OK; i++) code = w.pk_code[i];
  if (end == beg) code = C_EMPTY_JOB;
  g2a sa;
  sa.x = fp2_zero();
  sa.y = fp2_zero();
  uint32_t inf = 1;
  if (code == C_OK) {
    g2j s = w.rsig[beg];
    for (uint32_t i = beg + span; i < end; i += span) {  // jobs larger than the tree
      const g2j r = w.rsig[i];
      jac_add(s, s, r);
    }
    inf = jac_to_aff(sa, s) ? 0u : 1u;
  }
  w.s_aff[j] = sa;
  w.s_inf[j] = inf;
  w.job_code[j] = code;
}

// --------------------------------------------------------------- k_miller
// Work items: every job's sets taken two at a time (one shared Fp12
// accumulator and squaring per two pairs, miller_loop2), then one item per
// job for its (-G1, S_job) pair.  Item offsets per job come from a scan.
__global__ void BGV_BULK k_item_count(dev_batch b, dev_work w) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  const uint32_t lo = b.job_off[j], hi = b.job_off[j + 1];
  w.item_off[j] = hi > lo ? (hi - lo + b.pairs_per_item - 1) / b.pairs_per_item : 0u;
}

__global__ void BGV_BULK k_item_job(dev_batch b, dev_work w) {
  const uint32_t j = gtid();
  if (j >= b.n_jobs) return;
  for (uint32_t t = w.item_off[j]; t < w.item_off[j + 1]; t++) w.item_job[t] = j;
}

// k_miller (the set-pair Miller loops) lives in bgv_miller.hip (1 wave/SIMD).

// Cooperative variant (miller_coop.h): GROUPS pairs per 64-lane workgroup,
// 6 x SUB x HALF lanes per pair; pair t < n_sets is (r_t PK_t, H(m_t)), then
// (-G1, S_job).
template <int SUB, int HALF>
__global__ void __launch_bounds__(64, BGV_WAVES) k_miller_coop(dev_batch b, dev_work w, uint32_t first, uint32_t count) {
  using cfg = coop_cfg<SUB, HALF>;
  __shared__ coop_grp_t<SUB, HALF> sm[cfg::GROUPS];
  const uint32_t lane = threadIdx.x, grp = lane / cfg::LANES;
  const uint32_t r = lane % cfg::LANES;
  const uint32_t k = r / (SUB * HALF), h = (r / SUB) % HALF, q = r % SUB;
  const uint32_t t = first + blockIdx.x * cfg::GROUPS + grp;
  const bool in_range = grp < cfg::GROUPS && t < first + count;
  bool active = in_range;
  if (in_range) {
    g1a P;
    g2a Q;
    if (t < b.n_sets) {
      // set pairs run before the signatures are decoded (ST_MILLER overlaps
      // ST_SIG_SCALE): a job with a bad signature is rejected by its code and
      // its Miller values are never used
      active = w.pk_code[t] == C_OK;
      P = w.rpk_aff[t];
      Q = w.h_aff[t];
    } else {
      const uint32_t j = t - b.n_sets;
      active = w.job_code[j] == C_OK && !w.s_inf[j];
      P.x = G1_X_MONT;
      P.y = G1_NEG_Y_MONT;
      Q = w.s_aff[j];
    }
    if (active && k == 0 && q == 0 && h == 0) {
      coop_grp_t<SUB, HALF>& g = sm[grp];
      g.T[0] = Q.x;
      g.T[1] = Q.y;
      g.T[2] = fp2_one();
      g.Q[0] = Q.x;
      g.Q[1] = Q.y;
      g.px.c0 = P.x;
      fp_set_zero(g.px.c1);
      g.py.c0 = P.y;
      fp_set_zero(g.py.c1);
    }
  }
  __syncthreads();
  coop_miller<SUB, HALF>(sm[grp < cfg::GROUPS ? grp : 0], k, h, q, active);
  if (in_range && q == 0 && h == 0) {
    fp2_t v;
    if (active) v = sm[grp].f[k];
    else v = k == 0 ? fp2_one() : fp2_zero();  // skipped pair contributes 1
    fp2_t* dst = reinterpret_cast<fp2_t*>(&w.f_set[t]) + (k & 1) * 3 + (k >> 1);
    *dst = v;
  }
}

// per-set batch scalars (rng.h): one ChaCha20 block per set
struct chacha_key { uint32_t key[8], nonce[3]; };
__global__ void __launch_bounds__(64) k_gen_scalars(chacha_key k, uint64_t* out, uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  out[i] = batch_scalar(k.key, i, k.nonce);
}

// set codes for the host: signature code first, then the pubkey code
__global__ void BGV_BULK k_set_codes(dev_batch b, dev_work w) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  const int32_t c = w.sig_code[i];
  w.set_code[i] = c != C_OK ? c : w.pk_code[i];
}

// Montgomery <-> plain limbs for Fp12 values crossing the host boundary
// (the host never touches the __constant__ curve tables)
__global__ void BGV_BULK k_fp12_convert(const fp12_t* in, fp12_t* out, uint32_t n, uint32_t to_mont) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const fp_t* a = (const fp_t*)&in[i];
  fp_t* r = (fp_t*)&out[i];
  for (int k = 0; k < 12; k++) {
    fp_t t = a[k];
    if (to_mont) fp_to_mont(t, t);
    else fp_from_mont(t, t);
    r[k] = t;
  }
}

// ======================================================= synthetic data
// scalar field order r (little-endian u32)
BGV_CONST uint32_t FR_R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                              0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};

BGV_HD bool u256_ge_r(const uint32_t a[8]) {
  for (int i = 7; i >= 0; i--) {
    if (a[i] > FR_R[i]) return true;
    if (a[i] < FR_R[i]) return false;
  }
  return true;
}

BGV_HD void u256_sub_r(uint32_t a[8]) {
  uint32_t borrow = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a[i] - FR_R[i] - borrow;
    a[i] = (uint32_t)d;
    borrow = (uint32_t)(d >> 63);
  }
}

// a = (a + b) mod r, both < r
BGV_HD void fr_add(uint32_t a[8], const uint32_t b[8]) {
  uint32_t c = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a[i] + b[i] + c;
    a[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  if (u256_ge_r(a)) u256_sub_r(a);
}

// [k]P, k = 256-bit little-endian u32 words, left-to-right double-and-add
template <class F>
BGV_NI void jac_mul_u256(jac_t<F>& r, const jac_t<F>& p, const uint32_t k[8]) {
  jac_t<F> acc;
  jac_set_inf(acc);
  for (int w = 7; w >= 0; w--) {
    for (int bit = 31; bit >= 0; bit--) {
      jac_dbl(acc, acc);
      if ((k[w] >> bit) & 1u) jac_add(acc, acc, p);
    }
  }
  r = acc;
}

// PublicKey.fromBytes(pk, affine, validate=true) for untrusted keys
// (processDeposit.ts:59): decode + on-curve, infinity -> BLST_PK_IS_INFINITY,
// then the definitional subgroup test [r]P = O (once per deposit, so the
// 255 doublings are not worth an endomorphism shortcut)
__global__ void BGV_BULK k_pk_validate(const uint8_t* in, uint32_t n, int32_t* codes) {
  const uint32_t t = gtid();
  if (t >= n) return;
  g1a a;
  bool inf = false;
  int32_t c = g1_decompress(a, inf, in + 48u * t);
  if (c == C_OK && inf) c = C_PK_IS_INFINITY;
  if (c == C_OK) {
    g1j p, q;
    p.x = a.x;
    p.y = a.y;
    fe_one(p.z);
    jac_mul_u256(q, p, FR_R);
    if (!jac_is_inf(q)) c = C_POINT_NOT_IN_GROUP;
  }
  codes[t] = c;
}

// sk_i = SHA256("bgv-sk" || LE64(seed) || LE32(i)) (big-endian integer) mod r
__device__ void gen_sk(uint32_t sk[8], uint64_t seed, uint32_t i) {
  uint32_t blk[16];
  blk_clear(blk);
  const char tag[6] = {'b', 'g', 'v', '-', 's', 'k'};
  int pos = 0;
  for (int k = 0; k < 6; k++) blk_put(blk, pos++, (uint8_t)tag[k]);
  for (int k = 0; k < 8; k++) blk_put(blk, pos++, (uint32_t)(seed >> (8 * k)));
  for (int k = 0; k < 4; k++) blk_put(blk, pos++, (i >> (8 * k)));
  blk_put(blk, pos, 0x80);
  blk[15] = (uint32_t)pos * 8u;  // 18 bytes
  uint32_t st[8];
  for (int k = 0; k < 8; k++) st[k] = SHA256_IV[k];
  sha256_compress(st, blk);
  // digest words are big-endian: st[0] is the most significant
  for (int k = 0; k < 8; k++) sk[k] = st[7 - k];
  while (u256_ge_r(sk)) u256_sub_r(sk);
}

__global__ void BGV_BULK k_gen_keys(g1a* table, uint32_t* sk_store, uint32_t first, uint32_t n,
                                                 uint64_t seed) {
  const uint32_t t = gtid();
  if (t >= n) return;
  const uint32_t i = first + t;
  uint32_t sk[8];
  gen_sk(sk, seed, i);
  for (int k = 0; k < 8; k++) sk_store[8u * i + k] = sk[k];
  g1j g, p;
  g.x = G1_X_MONT; g.y = G1_Y_MONT; fe_one(g.z);
  jac_mul_u256(p, g, sk);
  g1a a;
  jac_to_aff(a, p);
  table[i] = a;
}

BGV_NI void g2_compress(uint8_t* out, const g2j& p) {
  g2a a;
  if (!jac_to_aff(a, p)) {
    for (int k = 0; k < 96; k++) out[k] = 0;
    out[0] = 0xc0;
    return;
  }
  uint8_t buf[96];
  fp_t t;
  fp_from_mont(t, a.x.c1);
  fp_to_be48(buf, t);
  fp_from_mont(t, a.x.c0);
  fp_to_be48(buf + 48, t);
  buf[0] |= 0x80u | (fp2_lex_largest(a.y) ? 0x20u : 0u);
  for (int k = 0; k < 96; k++) out[k] = buf[k];
}

__global__ void BGV_BULK k_gen_sign(dev_batch b, const uint32_t* sk_store, uint8_t* sigs_out) {
  const uint32_t i = gtid();
  if (i >= b.n_sets) return;
  uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t k = b.pk_off[i]; k < b.pk_off[i + 1]; k++) {
    const uint32_t idx = b.pk_idx[k];
    if (idx >= b.table_n) continue;
    uint32_t sk[8];
    for (int q = 0; q < 8; q++) sk[q] = sk_store[8u * idx + q];
    fr_add(s, sk);
  }
  uint8_t m[32];
  for (int k = 0; k < 32; k++) m[k] = b.msgs[32u * i + k];
  g2j h, sig;
  hash_to_g2(h, m);
  jac_mul_u256(sig, h, s);
  g2_compress(sigs_out + 192u * i, sig);
}

// ===================================================== field self-test
// bgv_debug_fp_ops: the device's modular additions (the inline-asm chains of
// fp_asm.h and their single / dual / lazy forms) on host-chosen operands,
// limbs in and out as they are (add and sub mod p do not care about the
// Montgomery form).  out[FP_OPS_N * i + k], k as in include/bgv.h.
__global__ void BGV_BULK k_fp_ops(const fp_t* ab, fp_t* out, uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const fp_t a = ab[2 * i], b = ab[2 * i + 1];
  fp_t* o = out + 13u * i;
  fp_t r0, r1;
  fp_add(r0, a, b); o[0] = r0;
  fp_sub(r0, a, b); o[1] = r0;
  fp_add2(r0, a, b, r1, b, b); o[2] = r0; o[3] = r1;
  fp_sub2(r0, a, b, r1, b, a); o[4] = r0; o[5] = r1;
  fp_add_sub(r0, a, b, r1, a, b); o[6] = r0; o[7] = r1;
  fp_add_lazy2(r0, a, b, r1, a, a); o[8] = r0; o[9] = r1;
  fp_neg(r0, a); o[10] = r0;
  fp_addnr_sub(r0, a, b, r1, b, a); o[11] = r0; o[12] = r1;
}

// bgv_debug_g2_decode: Signature.fromBytes' decode alone (g2_decompress /
// g2_deserialize, no subgroup check) on host-chosen encodings, so a test can
// put lanes that take the y.c1 = 0 / y.c0 = 0 arms of fp2_sqrt and
// fp2_lex_largest beside ordinary lanes of one wave and compare every decoded
// point (an off-subgroup point is zeroed by the verify path's k_sig).
__global__ void BGV_BULK k_g2_decode_dbg(const uint8_t* sigs192, const uint32_t* sig_len, uint8_t* out192, int32_t* codes,
                                        uint32_t n) {
  const uint32_t i = gtid();
  if (i >= n) return;
  const uint32_t len = sig_len[i];
  const uint8_t* s = sigs192 + 192u * i;
  g2a a;
  bool inf = false;
  int32_t code;
  if (len == 96u) code = g2_decompress(a, inf, s);
  else if (len == 192u) code = g2_deserialize(a, inf, s);
  else code = C_INVALID_SIZE;
  if (code != C_OK || inf) { a.x = fp2_zero(); a.y = fp2_zero(); }
  const fp_t* c[4] = {&a.x.c0, &a.x.c1, &a.y.c0, &a.y.c1};
  for (int k = 0; k < 4; k++) {
    fp_t t;
    fp_from_mont(t, *c[k]);
    fp_to_be48(out192 + 192u * i + 48 * k, t);
  }
  codes[i] = code;
}

// ========================================================= microbenchmarks
__global__ void __launch_bounds__(256) k_bench_fpmul(fp_t* io, uint32_t iters) {
  const uint32_t i = gtid();
  fp_t x = io[2 * i], y = io[2 * i + 1];
  for (uint32_t k = 0; k < iters; k++) fp_mul(x, x, y);
  io[2 * i] = x;
}

__global__ void __launch_bounds__(256) k_bench_mad(uint64_t* io, uint32_t iters) {
  const uint32_t i = gtid();
  uint64_t a0 = io[i], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t m = (uint32_t)a0 | 1u;
  for (uint32_t k = 0; k < iters; k++) {
    a0 = (uint64_t)(uint32_t)a0 * m + (a0 >> 32);
    a1 = (uint64_t)(uint32_t)a1 * m + (a1 >> 32);
    a2 = (uint64_t)(uint32_t)a2 * m + (a2 >> 32);
    a3 = (uint64_t)(uint32_t)a3 * m + (a3 >> 32);
    a4 = (uint64_t)(uint32_t)a4 * m + (a4 >> 32);
    a5 = (uint64_t)(uint32_t)a5 * m + (a5 >> 32);
    a6 = (uint64_t)(uint32_t)a6 * m + (a6 >> 32);
    a7 = (uint64_t)(uint32_t)a7 * m + (a7 >> 32);
  }
  io[i] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// ============================================================= launchers
static inline dim3 grid64(uint32_t n) { return dim3((n + 63u) / 64u); }

#define BGV_LAUNCH(k, n, ...)                                                 \
  do {                                                                        \
    if ((n) > 0) hipLaunchKernelGGL(k, grid64(n), dim3(64), 0, st, __VA_ARGS__); \
  } while (0)

void launch_raw_pks(hipStream_t st, const uint8_t* raw, g1a* out, uint32_t n) { BGV_LAUNCH(k_raw_pks, n, raw, out, n); }
void launch_table_from_compressed(hipStream_t st, const uint8_t* in, g1a* out, uint32_t n, int32_t* codes) {
  BGV_LAUNCH(k_table_from_compressed, n, in, out, n, codes);
}
void launch_table_from_uncompressed(hipStream_t st, const uint8_t* in, g1a* out, uint32_t n, int32_t* codes) {
  BGV_LAUNCH(k_table_from_uncompressed, n, in, out, n, codes);
}
void launch_export_g1a(hipStream_t st, const g1a* in, uint8_t* out96, uint32_t n) { BGV_LAUNCH(k_export_g1a, n, in, out96, n); }
void launch_export_g2a(hipStream_t st, const g2a* in, uint8_t* out192, uint32_t n) { BGV_LAUNCH(k_export_g2a, n, in, out192, n); }
void launch_pk_validate(hipStream_t st, const uint8_t* in, uint32_t n, int32_t* codes) {
  BGV_LAUNCH(k_pk_validate, n, in, n, codes);
}
void launch_table_export(hipStream_t st, const g1a* tab, uint8_t* out, uint32_t n) {
  BGV_LAUNCH(k_table_export, n, tab, out, n);
}
// Index-only set-up of ST_PK (balanced 32-key chunks) and ST_MILLER (work
// items): launched before the stages fork onto their streams, while the GPU
// is idle.  Under the bulk kernels the one-workgroup scan is starved of its
// CU (rocprofv3: 20 ms instead of tens of microseconds).
// the latency mode's hash maps, launched by prepare() before the host-side
// set-up of the batch (bgv_api.hip early_maps): they read only the messages
void launch_hash_maps(hipStream_t st, const dev_batch& b, const dev_work& w) {
  BGV_LAUNCH(k_hash_map, 2u * b.n_sets, b, w);
}

void launch_prep(hipStream_t st, const dev_batch& b, const dev_work& w) {
  BGV_LAUNCH(k_chunk_count, b.n_sets, b, w);
  if (b.n_sets) hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, w.chunk_off, b.n_sets);
  BGV_LAUNCH(k_chunk_set, b.n_sets, b, w);
  if (!b.miller_coop || b.miller_kv) {
    BGV_LAUNCH(k_item_count, b.n_jobs, b, w);
    if (b.n_jobs) hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, w.item_off, b.n_jobs);
    BGV_LAUNCH(k_item_job, b.n_jobs, b, w);
  }
}

// pairs [first, first + count) through the cooperative layout of `lanes`
// lanes per pair (6, 18 or 36)
static void launch_miller_coop(hipStream_t st, uint32_t lanes, const dev_batch& b, const dev_work& w, uint32_t first,
                               uint32_t count) {
  if (!count) return;
  if (lanes == 6) {
    constexpr uint32_t G = coop_cfg<1, 1>::GROUPS;
    hipLaunchKernelGGL((k_miller_coop<1, 1>), dim3((count + G - 1) / G), dim3(64), 0, st, b, w, first, count);
  } else if (lanes == 18) {
    constexpr uint32_t G = coop_cfg<3, 1>::GROUPS;
    hipLaunchKernelGGL((k_miller_coop<3, 1>), dim3((count + G - 1) / G), dim3(64), 0, st, b, w, first, count);
  } else {
    constexpr uint32_t G = coop_cfg<3, 2>::GROUPS;
    hipLaunchKernelGGL((k_miller_coop<3, 2>), dim3((count + G - 1) / G), dim3(64), 0, st, b, w, first, count);
  }
}

void launch_sig_check(hipStream_t st, const dev_batch& b, const dev_work& w) {
  // k_sig_split's check blocks only, for the sets from defer_from on
  const uint32_t nd = (b.n_sets - b.defer_from + 63u) / 64u;
  if (nd) hipLaunchKernelGGL(k_sig_split, dim3(nd), dim3(64), 0, st, b, w);
}

void launch_sig_fixup(hipStream_t st, const dev_batch& b, const dev_work& w) {
  BGV_LAUNCH(k_sig_fix, b.n_sets, b, w);
  BGV_LAUNCH(k_job_recode, b.n_jobs, b, w);
}

void launch_stage(hipStream_t st, int stage, const dev_batch& b, const dev_work& w) {
  const uint32_t span = 1u << b.span_log2;
  switch (stage) {
    case ST_SIG:
      if (b.split && !b.msm) {
        BGV_LAUNCH(k_sig_dec, b.n_sets, b, w);
        if (b.n_sets) {
          if (BGV_COOP_G2)
            launch_sig_split_coop(st, b, w);  // bgv_latency.hip
          else
            hipLaunchKernelGGL(k_sig_split, dim3(2u * ((b.n_sets + 63u) / 64u)), dim3(64), 0, st, b, w);
        }
        BGV_LAUNCH(k_sig_fix, b.n_sets, b, w);
      } else if (b.defer_grp && b.defer_from == 0) {
        BGV_LAUNCH(k_sig_dec, b.n_sets, b, w);  // subgroup check later: launch_sig_check
      } else {
        BGV_LAUNCH(k_sig, b.n_sets, b, w);
      }
      break;
    case ST_HASH:
      if (b.split) {
        if (!b.maps_early) BGV_LAUNCH(k_hash_map, 2u * b.n_sets, b, w);
        if (b.clear_lanes == 3) {
          launch_hash_clear_trio(st, b, w);  // bgv_latency.hip
        } else if (BGV_COOP_G2 && b.clear_lanes != 1) {
          launch_hash_clear_coop(st, b, w);  // bgv_latency.hip
        } else {
          BGV_LAUNCH(k_hash_clear, b.n_sets, b, w);
        }
      } else {
        BGV_LAUNCH(k_hash, b.n_sets, b, w);
      }
      break;
    case ST_PK:  // after launch_prep: the gather from the HBM table
      launch_pk_gather(st, b, w);  // bgv_gather.hip
      break;
    case ST_PK_SCALE:
      // latency mode: three lanes per set (bgv_latency.hip k_pk_coop)
      if (b.split && BGV_PK_COOP && b.n_sets < PK_COOP_MAX) launch_pk_coop(st, b, w);
      else BGV_LAUNCH(k_pk, b.n_sets, b, w);
      break;
    case ST_SIG_SCALE:
      if (b.split && !b.msm) break;  // [r_i] sigma_i already ran in k_sig_split
      if (b.msm == 2) {
        BGV_LAUNCH(k_msm_bucket, b.n_jobs * 16u, b, w);
      } else if (b.msm == 4) {
        BGV_LAUNCH(k_msm_digit, b.n_jobs * 256u, b, w);
      } else if (b.msm == 1) {
        if (b.n_jobs) {
          const uint32_t chunk = 1u << min(b.span_log2, 8u);  // LDS for one chunk of signatures
          hipLaunchKernelGGL(k_msm_fused, dim3(b.n_jobs), dim3(MSM_LANES), chunk * sizeof(g2a), st, b, w, chunk);
        }
      } else {
        BGV_LAUNCH(k_sig_scale, b.n_sets, b, w);
      }
      break;
    case ST_S_TREE:
      BGV_LAUNCH(k_set_job, b.n_jobs, b, w);
      if (b.msm == 2 || b.msm == 4) {
        if (b.msm == 2) BGV_LAUNCH(k_msm_window, b.n_jobs * 16u, b, w);
        // the window combination on nine lanes per job (bgv_latency.hip) in
        // the latency mode; bulk batches keep the 16-lane one-lane form
        if ((b.msm == 4 && BGV_MSM_JOB_COOP) || (b.msm == 2 && BGV_MSM_JOB_COOP_BULK))
          launch_msm_job_coop(st, b, w);
        else
          BGV_LAUNCH(k_msm_job, b.n_jobs * 16u, b, w);
        break;
      }
      if (b.msm == 1) {
        BGV_LAUNCH(k_job_code, b.n_jobs, b, w);
        break;
      }
      // nine lanes per addition while the first level's groups fit the SIMDs
      for (uint32_t s = 1; s < span; s *= 2) {
        if (BGV_COOP_G2 && b.n_sets < S_COOP_MAX) launch_s_level_coop(st, b, w, s);  // bgv_latency.hip
        else BGV_LAUNCH(k_s_level, b.n_sets, b, w, s);
      }
      BGV_LAUNCH(k_job_s, b.n_jobs, b, w, span);
      break;
    case ST_MILLER:  // (r_i PK_i, H(m_i)) pairs: needs ST_HASH and ST_PK only
      if (b.miller_kv) {
        launch_miller_kv(st, b, w);  // bgv_miller.hip
        break;
      }
      if (b.miller_coop == 2) {
        launch_miller_duo(st, b, w);  // bgv_miller.hip
        break;
      }
      if (b.miller_coop == 4) {
        launch_miller_quad(st, b, w);  // bgv_miller.hip
        break;
      }
      if (b.miller_coop) {
        if (b.n_sets)
          launch_miller_coop(st, b.miller_coop, b, w, 0u, b.n_sets);
        break;
      }
      launch_miller(st, b, w);  // bgv_miller.hip
      break;
    case ST_MILLER_JOBS:  // (-G1, S_job) pairs: needs ST_S_TREE
      // always the cooperative loop: one pair per job is latency-bound (a lone
      // lane takes ~19 ms at C4, the cooperative loop ~5 ms) and its waves
      // fit on the SIMDs the set-pair kernel leaves free
      if (b.n_jobs)
        launch_miller_coop(st, b.job_lanes, b, w, b.n_sets, b.n_jobs);
      break;
    case ST_F_TREE:
      launch_fp12_tail(st, stage, b, w);  // bgv_tail.hip
      break;
    case ST_BATCH_PROD:
      launch_fp12_tail(st, stage, b, w);
      break;
    case ST_BATCH_FINAL:
    case ST_JOB_FINAL: launch_fp12_tail(st, stage, b, w); break;
    case ST_SET_CODES: BGV_LAUNCH(k_set_codes, b.n_sets, b, w); break;
    default: break;
  }
}

void launch_fp12_convert(hipStream_t st, const fp12_t* in, fp12_t* out, uint32_t n, bool to_mont) {
  BGV_LAUNCH(k_fp12_convert, n, in, out, n, to_mont ? 1u : 0u);
}
void launch_gen_scalars(hipStream_t st, const uint32_t key[8], const uint32_t nonce[3], uint64_t* out, uint32_t n) {
  chacha_key k;
  for (int i = 0; i < 8; i++) k.key[i] = key[i];
  for (int i = 0; i < 3; i++) k.nonce[i] = nonce[i];
  BGV_LAUNCH(k_gen_scalars, n, k, out, n);
}
void launch_gen_keys(hipStream_t st, g1a* table, uint32_t* sk, uint32_t first, uint32_t n, uint64_t seed) {
  BGV_LAUNCH(k_gen_keys, n, table, sk, first, n, seed);
}
void launch_gen_sign(hipStream_t st, const dev_batch& b, const uint32_t* sk, uint8_t* out) {
  BGV_LAUNCH(k_gen_sign, b.n_sets, b, sk, out);
}
void launch_g2_decode_dbg(hipStream_t st, const uint8_t* sigs192, const uint32_t* sig_len, uint8_t* out192, int32_t* codes,
                         uint32_t n) {
  BGV_LAUNCH(k_g2_decode_dbg, n, sigs192, sig_len, out192, codes, n);
}
void launch_fp_ops(hipStream_t st, const fp_t* ab, fp_t* out, uint32_t n) {
  if (n) hipLaunchKernelGGL(k_fp_ops, dim3((n + 63u) / 64u), dim3(64), 0, st, ab, out, n);
}
void launch_bench_fpmul(hipStream_t st, fp_t* io, uint32_t lanes, uint32_t iters) {
  hipLaunchKernelGGL(k_bench_fpmul, dim3(lanes / 256), dim3(256), 0, st, io, iters);
}
void launch_bench_mad(hipStream_t st, uint64_t* io, uint32_t lanes, uint32_t iters) {
  hipLaunchKernelGGL(k_bench_mad, dim3(lanes / 256), dim3(256), 0, st, io, iters);
}

}  // namespace bgv
