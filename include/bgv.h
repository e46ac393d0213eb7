/*
 * bgv.h -- C ABI of the MI355X (gfx950) BLS12-381 signature-set batch
 * verifier ("bgv" = BLS GPU verifier).
 *
 * This is the drop-in boundary for the hot path of
 *   IBlsVerifier.verifySignatureSets(sets, opts)
 *   (packages/beacon-node/src/chain/bls/interface.ts:20-51)
 * in maschad/lodestar.  Every entry point below names the reference
 * interface it replaces.  Plain pointers and sizes only; no torch / HIP
 * types appear in the signatures.  All functions return 0 (BGV_OK) on
 * success or a negative BGV_E* status; per-set verification outcomes are
 * reported as the positive blst error codes listed in bgv_set_code.
 *
 * Threading: a bgv_ctx owns one HIP device and one stream.  Calls on one
 * context must be serialised by the caller (the N-API / Python host layers
 * do this); different contexts may be used from different threads.
 */
#ifndef BGV_H
#define BGV_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BGV_ABI_VERSION 4

/* ---- status of an API call (negative) ---------------------------------- */
enum bgv_status {
  BGV_OK = 0,
  BGV_E_INVALID_ARG = -1,
  BGV_E_HIP = -2,          /* HIP runtime error (device missing, OOM, fault) */
  BGV_E_NO_DEVICE = -3,
  BGV_E_TABLE_RANGE = -4,  /* pubkey index outside the resident table */
  BGV_E_EMPTY_SET = -5,    /* a set with zero pubkeys (EMPTY_AGGREGATE_ARRAY) */
  BGV_E_BAD_PUBKEY = -6,   /* bgv_pubkeys_set: a key does not deserialize (the
                              text names the key and its BLST_* code) */
  BGV_E_STATE = -7,        /* bgv_partial_finish without a preceding bgv_partial */
};

/* ---- per-set / per-job outcome codes (>= 0) ------------------------------
 * Numbering follows blst's BLST_ERROR enum (the codes @chainsafe/blst turns
 * into "BLST_ERROR: BLST_<NAME>" exceptions), plus the size condition
 * @chainsafe/blst raises before reaching blst and a range guard for
 * device-resident index lists.                                             */
enum bgv_set_code {
  BGV_SET_OK = 0,
  BGV_SET_BAD_ENCODING = 1,
  BGV_SET_POINT_NOT_ON_CURVE = 2,
  BGV_SET_POINT_NOT_IN_GROUP = 3,
  BGV_SET_AGGR_TYPE_MISMATCH = 4,
  BGV_SET_VERIFY_FAIL = 5,
  BGV_SET_PK_IS_INFINITY = 6,
  BGV_SET_BAD_SCALAR = 7,
  BGV_SET_INVALID_SIZE = 8,
  BGV_SET_INDEX_RANGE = 9, /* device batch named a pubkey index >= table size */
};

/* job verdicts written to job_result[] */
enum bgv_job_result {
  BGV_JOB_INVALID = 0, /* encodings fine, pairing check failed -> resolve(false) */
  BGV_JOB_VALID = 1,   /* every set verified                  -> resolve(true)  */
  /* negative: -(bgv_set_code) of the first set (in set order) that could not
   * be parsed / validated -> reject(Error("BLST_ERROR: BLST_<NAME>"))       */
};

/* pubkey wire formats accepted by bgv_pubkeys_set */
enum bgv_pk_format {
  BGV_PK_COMPRESSED_48 = 0,   /* ZCash compressed G1, as in BeaconState.validators */
  BGV_PK_UNCOMPRESSED_96 = 1, /* x||y big-endian; PointFormat.uncompressed
                                 (multithread/index.ts:132,177) */
};

typedef struct bgv_ctx bgv_ctx;

/* One device batch = n_sets signature sets grouped into n_jobs jobs.  A job
 * is what the reference hands to verifySignatureSetsMaybeBatch
 * (chain/bls/maybeBatch.ts:16-38): its verdict is the AND of its sets.
 * Sets of one job are contiguous: job j owns sets [job_offsets[j],
 * job_offsets[j+1]).
 *
 * Pubkeys arrive as index lists into the HBM-resident index2pubkey table
 * (state-transition/src/cache/pubkeyCache.ts:6) instead of serialized
 * points: set i aggregates table entries pk_indices[pk_offsets[i] ..
 * pk_offsets[i+1]).  An index with bit 31 set selects entry
 * (index & 0x7fffffff) of raw_pks instead (pubkeys not in the table, e.g.
 * BLS-to-execution changes, signatureSets/blsToExecutionChange.ts:32).
 * An index past the table (or past n_raw) rejects only its job, with set
 * code BGV_SET_INDEX_RANGE: the reference fails such a lookup on the caller's
 * side (index2pubkey[i] is undefined), so other co-batched jobs are unaffected.
 * A set with no pubkeys fails the whole call with BGV_E_EMPTY_SET (callers
 * reject EMPTY_AGGREGATE_ARRAY before batching, chain/bls/utils.ts:11).
 * Host batches are copied into pinned staging memory first and every
 * contract check runs on that copy, so a caller that mutates its arrays
 * during the call cannot make the device read out of bounds.  On-device
 * batches (on_device = 1) are trusted to satisfy the contract: offsets
 * monotone, job_offsets spanning [0, n_sets], pk_indices as long as
 * pk_offsets[n_sets].
 *
 * Signatures: sig_len[i] bytes at sigs + 192*i (96 = compressed,
 * 192 = uncompressed; any other length yields BGV_SET_INVALID_SIZE, the
 * reference's "BLST_INVALID_SIZE", e2e/chain/bls/multithread.test.ts:97).
 *
 * scalars: 64-bit non-zero random multipliers, one per set (blst
 * mul_n_aggregate randomness).  NULL = drawn inside the library
 * (production): ChaCha20 on the device, keyed per call by 32 bytes of
 * getrandom().  Tests inject them for reproducibility.
 *
 * When `on_device` is non-zero every array pointer is a device pointer on
 * the context's device (inputs already resident in HBM); otherwise they are
 * host pointers and the library stages them.  The library works on its own
 * streams: every write to a device-resident input (and to an output buffer
 * such as bgv_gen_sign's sigs_out) must be complete before the call, e.g.
 * the producing stream synchronized (lodestar_amd/native.py does this for
 * torch tensors).                                                         */
typedef struct bgv_batch {
  uint32_t n_sets;
  uint32_t n_jobs;
  const uint32_t* job_offsets; /* [n_jobs + 1] */
  const uint32_t* pk_offsets;  /* [n_sets + 1] */
  const uint32_t* pk_indices;  /* [pk_offsets[n_sets]] */
  const uint8_t* raw_pks;      /* [n_raw][96] uncompressed big-endian, may be NULL */
  uint32_t n_raw;
  const uint8_t* msgs;         /* [n_sets][32] signing roots */
  const uint8_t* sigs;         /* [n_sets][192] */
  const uint32_t* sig_len;     /* [n_sets] */
  const uint64_t* scalars;     /* [n_sets] or NULL */
  uint32_t on_device;
} bgv_batch;

/* Timings of the last bgv_verify call (ms, HIP events around each stage on
 * the stream it ran on; stages 0-3 run concurrently on three streams, so their
 * times overlap and total_ms is less than their sum) plus the counters the reference pool exports as
 * lodestar_bls_thread_pool_* metrics (metrics/metrics/lodestar.ts:350-430). */
#define BGV_N_STAGES 16
typedef struct bgv_stats {
  float stage_ms[BGV_N_STAGES]; /* see bgv_stage_name() */
  float total_ms;
  uint32_t batch_retries;       /* 1 when the whole-batch check failed */
  uint32_t batch_sigs_success;  /* sets accepted by the whole-batch check */
  uint32_t n_sets;
  uint32_t n_jobs;
  uint64_t pubkeys_aggregated;  /* lodestar_bls_aggregated_pubkeys_total */
  /* the pipeline variant the batch ran with (chosen by batch size, or forced
   * by bgv_cfg); also filled by bgv_last_stats                              */
  uint32_t split;               /* 1: latency-mode hash and signature kernels */
  uint32_t miller_lanes;        /* set-pair Miller loop: lanes per pair (1 = one-lane loop) */
  uint32_t pairs_per_item;      /* one-lane loop: pairs sharing an accumulator */
  uint32_t msm;                 /* sum r_i sigma_i variant (bgv_cfg.msm) */
  uint32_t lines;               /* 1: fixed-argument Miller lines */
  uint32_t defer_from;          /* subgroup checks of sets >= defer_from run beside the Miller loops (n_sets: none) */
  uint32_t clear_lanes;         /* latency mode: lanes per point of the cofactor clearing */
  uint32_t miller_kv;           /* 0, or the product slots of the two-pair Miller loop in Karatsuba views (3 S lanes per two pairs) */
} bgv_stats;

/* Pipeline overrides for tests and A/B tools.  Production opens contexts with
 * bgv_open (every field "auto": the variant is chosen per batch by its size,
 * from measured sweeps).  No environment variable changes the pipeline.    */
typedef struct bgv_cfg {
  uint32_t struct_size; /* sizeof(bgv_cfg) */
  int32_t split;        /* -1 auto; 0 bulk kernels; 1 latency mode (two-lane hash maps, cooperative G2) */
  int32_t miller;       /* -1 auto; 1 one-lane set-pair loop; 2 / 4 two- / four-lane loop; 6 / 18 / 36 lanes per pair (cooperative) */
  int32_t job_lanes;    /* 0 auto (36); 6 / 18 / 36: lanes of the per-job (-G1, S_job) pairs */
  int32_t msm;          /* -1 auto; 0 per-set [r_i] sigma_i + tree; 1 per-job bucket MSM (one workgroup per job); 2 the (job, window)-lane MSM;
                           3 one-lane per-set [r_i] sigma_i + tree, subgroup checks deferred; 4 the (job, window, digit)-lane MSM */
  int32_t pairs;        /* 0 auto; 1 / 2 / 4 pairs per one-lane Miller work item (4: over precomputed lines only, else 2) */
  int32_t prefold;      /* -1 auto; 0 / 1 two-level per-job Miller fold */
  int32_t lines;        /* -1 auto; 0 / 1 fixed-argument lines (bulk mode, one-lane loop) */
  int32_t defer_pct;    /* -1 auto; 0..100: share of the G2 subgroup checks run beside the Miller loops (bulk mode) */
  int32_t timing;       /* -1 auto (batches >= 65,536 sets); 0 / 1 per-stage timing events */
  int32_t clear_lanes;  /* -1 auto; 1 / 3 / 9 lanes per point of the latency mode's cofactor clearing */
  int32_t miller_kv;    /* -1 auto; 0 off; 2 / 3 / 6 / 9: the two-pair Miller loop in Karatsuba views on 6 / 9 / 18 / 27 lanes per two pairs */
  int32_t cu_split;     /* 0: every CU of the device (default).  N > 0: a PRIORITY context whose streams run only
                           on N reserved CUs (the highest CU ids: with N = 8k, k CUs of every XCC), for
                           verifyOnMainThread single sets (multithread/index.ts:155-167) that must not wait for a
                           bulk batch's waves; N < 0: a bulk context whose streams leave those |N| CUs free (ABI 4) */
} bgv_cfg;
/* every field "auto" */
void bgv_cfg_default(bgv_cfg* cfg);

int bgv_abi_version(void);
/* SHA-256 (hex) of the sources this library was compiled from (csrc + this
 * header, tools/build.py source_hash); bindings refuse a library whose id
 * differs from the tree beside it, so a stale build is never run */
const char* bgv_build_id(void);
const char* bgv_set_code_name(int code); /* "BLST_BAD_ENCODING", ... */
const char* bgv_stage_name(int stage);
const char* bgv_last_error(void);        /* thread-local text of the last failure */

/* Open a context on HIP device `device` (chain/chain.ts:199-202 picks the
 * verifier at node start; this is the GPU branch's constructor, replacing
 * `new BlsMultiThreadWorkerPool(opts, modules)`, multithread/index.ts:120). */
int bgv_open(int device, bgv_ctx** out);
/* bgv_open with pipeline overrides (tests, A/B tools); cfg may be NULL */
int bgv_open_cfg(int device, const bgv_cfg* cfg, bgv_ctx** out);
/* BlsMultiThreadWorkerPool.close (multithread/index.ts:193-214) */
int bgv_close(bgv_ctx* ctx);

/* index2pubkey table management: mirrors syncPubkeys / addPubkey
 * (state-transition/src/cache/pubkeyCache.ts:56-77, cache/epochContext.ts:
 * 701-704).  Keys are trusted (validated at deposit, block/processDeposit.ts:
 * 57-66) and stored as affine Montgomery (x, y), 96 B per validator.
 * Like PublicKey.fromBytes(pk, jacobian) (no validation) a key must still
 * deserialize: flags, x < p, on the curve; otherwise the call fails with
 * BGV_E_BAD_PUBKEY and the table is unchanged.  The infinity key is stored
 * as the identity (a set aggregating only identities is BLST_PK_IS_INFINITY).
 * The table is append-only like syncPubkeys: first_index <= current count
 * (rows below the count may be rewritten, as addPubkey does); a gap fails
 * with BGV_E_TABLE_RANGE.  At most 2^31 - 1 rows (bit 31 of an index
 * selects raw_pks).                                                       */
int bgv_pubkeys_set(bgv_ctx* ctx, uint32_t first_index, uint32_t n, const uint8_t* data, uint32_t format);
int bgv_pubkeys_count(bgv_ctx* ctx, uint32_t* count);
/* read back entries as 96-byte uncompressed big-endian (tests, checkpoints) */
int bgv_pubkeys_get(bgv_ctx* ctx, uint32_t first_index, uint32_t n, uint8_t* out96);

/* Untrusted-key validation: bls.PublicKey.fromBytes(pk, CoordType.affine,
 * validate=true) for n 48-byte compressed keys, as deposits do once per new
 * validator (state-transition/src/block/processDeposit.ts:57-66; also
 * beacon-node/src/chain/validation/blobsSidecar.ts:129).  codes[i] is a
 * bgv_set_code: 0 valid, BAD_ENCODING (flags / x >= p), POINT_NOT_ON_CURVE,
 * PK_IS_INFINITY, POINT_NOT_IN_GROUP ([r]P != O).  Valid keys can then be
 * appended with bgv_pubkeys_set.                                          */
int bgv_pubkeys_validate(bgv_ctx* ctx, const uint8_t* pk48, uint32_t n, int32_t* codes);

/* Verify one device batch.  Replaces the worker body
 * verifyManySignatureSets (multithread/worker.ts:30-106) together with
 * verifySignatureSetsMaybeBatch (maybeBatch.ts:16-38) and the main-thread
 * aggregation getAggregatedPubkey (chain/bls/utils.ts:5-16):
 *   job_result[n_jobs]  (host memory) BGV_JOB_* per job;
 *   set_code[n_sets]    (host memory, may be NULL) bgv_set_code per set;
 *   stats               (may be NULL).
 * One whole-batch pairing check runs first; only when it fails is every
 * job checked on its own (the worker's per-job retry, worker.ts:74-85). */
int bgv_verify(bgv_ctx* ctx, const bgv_batch* batch, int32_t* job_result, int32_t* set_code, bgv_stats* stats);
/* Stage timings (stage_ms, total_ms) of the last pipeline run on the context
 * (bgv_verify, bgv_partial, bgv_partial_finish); counters are left zero. */
int bgv_last_stats(bgv_ctx* ctx, bgv_stats* stats);

/* Multi-GPU partials: run the batch up to, but excluding, the
 * final exponentiation and return this shard's Miller product (576 B, 12
 * Fp coefficients of w^0..w^5, c0||c1 each, 48-byte big-endian) with the
 * per-set codes and per-job provisional results (job_result may be NULL):
 * -code for a job rejected by a parse / subgroup / pubkey error (final),
 * 1 for every other job (valid iff the node's combined check passes).
 * ok_out = 1 when no job was rejected.  The shard's intermediates stay on
 * the context for bgv_partial_finish until the next call on it. */
int bgv_partial(bgv_ctx* ctx, const bgv_batch* batch, uint8_t* miller576, int32_t* set_code, int32_t* job_result,
                int32_t* ok_out);
/* Localisation after a failed combined check (SURVEY §8e "Failure"): the
 * final exponentiation of THIS shard's product, then per-job final
 * exponentiations only if it fails (the worker's per-job retry,
 * multithread/worker.ts:74-85), on the intermediates bgv_partial left.
 * job_result[n_jobs] as for bgv_verify.  BGV_E_STATE when the previous call
 * on the context was not bgv_partial. */
int bgv_partial_finish(bgv_ctx* ctx, int32_t* job_result, bgv_stats* stats);
/* Combine n partial Miller products and run ONE final exponentiation:
 * *is_one = 1 iff the product maps to 1 in GT. */
int bgv_combine_final(bgv_ctx* ctx, const uint8_t* millers576, uint32_t n, int32_t* is_one);

/* ---- test-only: per-stage intermediates (SURVEY §8c golden plan) --------
 * Runs bgv_verify on the batch and copies out the canonical values of every
 * stage.  Points are affine, plain big-endian: G1 x || y (96 B), G2
 * x.c0 || x.c1 || y.c0 || y.c1 (192 B); the identity and rejected entries
 * are all-zero.  GT values are 576 B as for bgv_partial and are the cube of
 * the textbook final exponentiation f^((p^12 - 1)/r) (the hard-part chain
 * computes 3 (p^4 - p^2 + 1)/r).  Any pointer may be NULL.
 *   pair_fe[n_sets + n_jobs]: FE of every Miller value: set pairs first
 *   (with P = 2 or 4 pairs per Miller work item, bgv_stats.pairs_per_item,
 *   the item's first entry, job offset + P k, holds the item's product and
 *   the other P - 1 the identity), then each job's (-G1, S_job) pair. */
typedef struct bgv_debug {
  uint8_t* sig_aff;  /* [n_sets][192] decoded signature (zero: invalid / identity) */
  uint8_t* h_aff;    /* [n_sets][192] H(m_i) */
  uint8_t* pk_agg;   /* [n_sets][96]  aggregated pubkey before the batch scalar */
  uint8_t* rpk_aff;  /* [n_sets][96]  r_i * aggregated pubkey */
  uint8_t* s_aff;    /* [n_jobs][192] S_job = sum over the job of r_i sigma_i */
  uint8_t* pair_fe;  /* [n_sets + n_jobs][576] */
  uint8_t* job_fe;   /* [n_jobs][576] FE of the job's Miller product */
  uint8_t* batch_fe; /* [576] FE of the whole-batch product */
} bgv_debug;
int bgv_debug_stages(bgv_ctx* ctx, const bgv_batch* batch, int32_t* job_result, int32_t* set_code, bgv_debug* out);

/* ---- synthetic workload generation (bench / tests; not on the verify path) */
/* table[first .. first+n) := sk_i * G1 with sk_i = SHA256("bgv-sk" || LE64(seed)
 * || LE32(i)) mod r; keeps sk on the device for bgv_gen_sign. */
int bgv_gen_keys(bgv_ctx* ctx, uint32_t first_index, uint32_t n, uint64_t seed);
/* sigs96[i] = compress((sum_{j in set i} sk_j mod r) * H(msgs[i])).
 * Pointers follow batch->on_device; sigs_out is in the same space. */
int bgv_gen_sign(bgv_ctx* ctx, const bgv_batch* batch, uint8_t* sigs_out192);

/* ---- field self-test (tests only) ---------------------------------------- */
/* The device's modular add/sub primitives on n operand pairs: ab_in holds
 * a_i || b_i as 2 x 12 little-endian u32 limbs (each < p; add and sub mod p
 * are independent of the Montgomery form), out receives BGV_FP_OPS_N
 * elements of 12 limbs per pair: a+b, a-b, [a+b, 2b] (dual add), [a-b, b-a]
 * (dual sub), [a+b, a-b] (add/sub pair), [a+b, 2a] unreduced (dual lazy
 * add), -a, [a+b unreduced, b-a] (lazy add / sub pair).  Host pointers. */
#define BGV_FP_OPS_N 13
int bgv_debug_fp_ops(bgv_ctx* ctx, const uint32_t* ab_in, uint32_t n, uint32_t* out);
/* The signature decode of Signature.fromBytes(sig, affine, true) without its
 * subgroup check (tests only; maybeBatch.ts:23,36): sigs192[i] holds a 96-byte
 * compressed or 192-byte uncompressed encoding (sig_len[i]); out192[i] gets the
 * affine point as x.c0 || x.c1 || y.c0 || y.c1, 48 big-endian bytes each
 * (zero for the identity or a failed decode), codes[i] the BGV set code.
 * Host pointers. */
int bgv_debug_g2_decode(bgv_ctx* ctx, const uint8_t* sigs192, const uint32_t* sig_len, uint32_t n, uint8_t* out192,
                        int32_t* codes);

/* ---- microbenchmarks for the roofline ------------------------ */
/* Montgomery Fp-mul throughput: `lanes` independent chains of `iters`
 * products; returns device ms (HIP events). */
int bgv_bench_fpmul(bgv_ctx* ctx, uint32_t lanes, uint32_t iters, float* ms);
/* raw v_mad_u64_u32 throughput: lanes * iters * 8 dependent-free mads */
int bgv_bench_mad(bgv_ctx* ctx, uint32_t lanes, uint32_t iters, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* BGV_H */
