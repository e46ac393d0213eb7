/* N-API addon over libbgv.so: the binding a Lodestar maintainer adds beside
 * chain/bls/multithread.  Plain C against
 * node_api.h (N-API v4+, Node >= 12), no node-addon-api / C++ wrapper.
 *
 *   abiVersion() -> number                      bgv_abi_version
 *   buildId() -> string                         bgv_build_id
 *   codeName(code) -> "BLST_..."                 bgv_set_code_name
 *   open(device, cuSplit = 0) -> ctx (external)  bgv_open_cfg  (multithread/index.ts:120); cuSplit N > 0:
 *                                                a priority context on N reserved CUs (verifyOnMainThread),
 *                                                N < 0: a bulk context that leaves them free (bgv_cfg.cu_split)
 *   close(ctx)                                   bgv_close     (multithread/index.ts:193-214)
 *   pubkeysSet(ctx, first, Uint8Array, format)   bgv_pubkeys_set (pubkeyCache.ts:56-77)
 *   pubkeysCount(ctx) -> number
 *   pubkeysValidate(ctx, Uint8Array) -> Int32Array   bgv_pubkeys_validate (processDeposit.ts:57-66)
 *   verify(ctx, batch) -> Promise<result>        bgv_verify on the libuv pool (worker.ts:30-106)
 *   verifySync(ctx, batch) -> result             BlsSingleThreadVerifier (blocks the calling thread)
 *   partial(ctx, batch) -> Promise<result + {miller: Uint8Array(576), ok}>
 *                                                bgv_partial: one shard of a multi-GPU batch
 *   combineFinal(ctx, Uint8Array(576 n)) -> Promise<boolean>
 *                                                bgv_combine_final: ONE final exponentiation of the shards
 *   partialFinish(ctx) -> Promise<result>        bgv_partial_finish: localise the last partial()'s shard
 *                                                after a failed combined check
 *
 * batch = {jobOffsets: Uint32Array, pkOffsets: Uint32Array, pkIndices:
 * Uint32Array, msgs: Uint8Array, sigs: Uint8Array (192 B per set), sigLen:
 * Uint32Array, rawPks?: Uint8Array (96 B per key)}.
 * result = {results: Int32Array (bgv_job_result per job: 1 valid, 0 invalid,
 * -code rejected), batchRetries, batchSigsSuccess, pubkeysAggregated,
 * deviceMs, workerStartMs, workerEndMs}: the BlsWorkResult fields
 * (multithread/types.ts:26-38) the pool's metrics are fed from.  For
 * partial() `results` is provisional: -code for a job rejected by a parse /
 * subgroup / pubkey error (final), 1 for every other job (valid iff the
 * combined check passes).  Contexts on different devices run their queued
 * work concurrently on the libuv pool (one pool thread per call in flight:
 * size UV_THREADPOOL_SIZE >= the device count, napi/index.js does).
 *
 * Ownership: the offset arrays are copied when the call
 * is made and every length is checked against the copies, so a caller that
 * mutates its typed arrays while the work is queued cannot make the library
 * read past them; the other arrays are pinned by references until the work
 * completes (the library copies them to pinned memory and HBM and keeps
 * nothing).  The context external is referenced by every queued work item,
 * so it outlives them.  A context is not thread-safe: calls on one context
 * are serialised by its mutex. */
#include <node_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "bgv.h"

#define NAPI_CALL(env, call)                                              \
  do {                                                                    \
    if ((call) != napi_ok) {                                              \
      napi_throw_error((env), NULL, "bgv addon: N-API call failed: " #call); \
      return NULL;                                                        \
    }                                                                     \
  } while (0)

typedef struct {
  bgv_ctx* ctx;
  pthread_mutex_t mu;
  int closed;
  uint32_t partial_jobs; /* job count of the last partial() (sizes partialFinish's results) */
} addon_ctx;

static void ctx_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  addon_ctx* c = (addon_ctx*)data;
  pthread_mutex_lock(&c->mu); /* no work item can hold the context here (each references it), but be exact */
  if (!c->closed) bgv_close(c->ctx);
  c->closed = 1;
  pthread_mutex_unlock(&c->mu);
  pthread_mutex_destroy(&c->mu);
  free(c);
}

static napi_value throw_bgv(napi_env env, int status) {
  char msg[512];
  snprintf(msg, sizeof msg, "bgv error %d: %s", status, bgv_last_error());
  napi_throw_error(env, NULL, msg);
  return NULL;
}

static addon_ctx* get_ctx(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "expected a bgv context");
    return NULL;
  }
  addon_ctx* c = (addon_ctx*)p;
  if (c->closed) {
    napi_throw_error(env, "QUEUE_ERROR_QUEUE_ABORTED", "QUEUE_ERROR_QUEUE_ABORTED: bgv context closed");
    return NULL;
  }
  return c;
}

/* typed-array view: data pointer and element count; -1 on type error */
static int typed(napi_env env, napi_value v, napi_typedarray_type want, void** data, size_t* len) {
  bool is = false;
  if (napi_is_typedarray(env, v, &is) != napi_ok || !is) return -1;
  napi_typedarray_type t;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok || t != want) return -1;
  return 0;
}

/* ------------------------------------------------------------------ sync */
static napi_value AbiVersion(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value r;
  NAPI_CALL(env, napi_create_int32(env, bgv_abi_version(), &r));
  return r;
}

static napi_value BuildId(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value r;
  NAPI_CALL(env, napi_create_string_utf8(env, bgv_build_id(), NAPI_AUTO_LENGTH, &r));
  return r;
}

static napi_value CodeName(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value a[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  int32_t code = 0;
  NAPI_CALL(env, napi_get_value_int32(env, a[0], &code));
  napi_value r;
  NAPI_CALL(env, napi_create_string_utf8(env, bgv_set_code_name(code), NAPI_AUTO_LENGTH, &r));
  return r;
}

static napi_value Open(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value a[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  int32_t dev = 0, cu_split = 0;
  if (argc >= 1) NAPI_CALL(env, napi_get_value_int32(env, a[0], &dev));
  if (argc >= 2) NAPI_CALL(env, napi_get_value_int32(env, a[1], &cu_split));
  bgv_cfg cfg;
  bgv_cfg_default(&cfg);
  cfg.cu_split = cu_split;
  bgv_ctx* ctx = NULL;
  const int st = bgv_open_cfg(dev, &cfg, &ctx);
  if (st != BGV_OK) return throw_bgv(env, st);
  addon_ctx* c = (addon_ctx*)calloc(1, sizeof *c);
  c->ctx = ctx;
  pthread_mutex_init(&c->mu, NULL);
  napi_value r;
  NAPI_CALL(env, napi_create_external(env, c, ctx_finalize, NULL, &r));
  return r;
}

static napi_value Close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value a[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  pthread_mutex_lock(&c->mu);  /* waits for in-flight work */
  c->closed = 1;
  bgv_close(c->ctx);
  pthread_mutex_unlock(&c->mu);
  return NULL;
}

static napi_value PubkeysSet(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value a[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  uint32_t first = 0, fmt = 0;
  NAPI_CALL(env, napi_get_value_uint32(env, a[1], &first));
  NAPI_CALL(env, napi_get_value_uint32(env, a[3], &fmt));
  void* data;
  size_t len;
  if (typed(env, a[2], napi_uint8_array, &data, &len)) {
    napi_throw_type_error(env, NULL, "pubkeys must be a Uint8Array");
    return NULL;
  }
  const size_t w = fmt == BGV_PK_UNCOMPRESSED_96 ? 96 : 48;
  pthread_mutex_lock(&c->mu);
  const int st = bgv_pubkeys_set(c->ctx, first, (uint32_t)(len / w), (const uint8_t*)data, fmt);
  pthread_mutex_unlock(&c->mu);
  if (st != BGV_OK) return throw_bgv(env, st);
  return NULL;
}

static napi_value PubkeysCount(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value a[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  uint32_t n = 0;
  pthread_mutex_lock(&c->mu);
  const int st = bgv_pubkeys_count(c->ctx, &n);
  pthread_mutex_unlock(&c->mu);
  if (st != BGV_OK) return throw_bgv(env, st);
  napi_value r;
  NAPI_CALL(env, napi_create_uint32(env, n, &r));
  return r;
}

static napi_value new_int32_array(napi_env env, const int32_t* src, size_t n) {
  void* dst = NULL;
  napi_value ab, arr;
  NAPI_CALL(env, napi_create_arraybuffer(env, 4 * n, &dst, &ab));
  if (n) memcpy(dst, src, 4 * n);
  NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, n, ab, 0, &arr));
  return arr;
}

static napi_value PubkeysValidate(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value a[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  void* data;
  size_t len;
  if (typed(env, a[1], napi_uint8_array, &data, &len)) {
    napi_throw_type_error(env, NULL, "pubkeys must be a Uint8Array of 48-byte keys");
    return NULL;
  }
  const uint32_t n = (uint32_t)(len / 48);
  int32_t* codes = (int32_t*)calloc(n ? n : 1, 4);
  pthread_mutex_lock(&c->mu);
  const int st = bgv_pubkeys_validate(c->ctx, (const uint8_t*)data, n, codes);
  pthread_mutex_unlock(&c->mu);
  if (st != BGV_OK) {
    free(codes);
    return throw_bgv(env, st);
  }
  napi_value r = new_int32_array(env, codes, n);
  free(codes);
  return r;
}

/* ----------------------------------------------------------------- verify */
enum { F_JOB, F_PKO, F_PKI, F_MSG, F_SIG, F_LEN, F_RAW, N_FIELDS };
static const char* FIELD[N_FIELDS] = {"jobOffsets", "pkOffsets", "pkIndices", "msgs", "sigs", "sigLen", "rawPks"};
static const napi_typedarray_type FIELD_T[N_FIELDS] = {napi_uint32_array, napi_uint32_array, napi_uint32_array,
                                                       napi_uint8_array,  napi_uint8_array,  napi_uint32_array,
                                                       napi_uint8_array};

enum { K_VERIFY, K_PARTIAL, K_FINISH, K_COMBINE };

typedef struct {
  int kind;
  addon_ctx* c;
  bgv_batch b;
  uint8_t miller[576];  /* K_PARTIAL */
  int32_t ok;           /* K_PARTIAL: no job rejected; K_COMBINE: the product is 1 in GT */
  uint8_t* parts;       /* K_COMBINE: a copy of the partials */
  uint32_t n_parts;
  uint32_t* job_off; /* copies made at call time (the library reads these) */
  uint32_t* pk_off;
  int32_t* job_result;
  bgv_stats stats;
  double t_start_ms, t_end_ms;
  int status;
  char err[512];
  napi_ref refs[N_FIELDS];
  napi_ref ctx_ref;
  napi_async_work work;
  napi_deferred deferred;
} verify_job;

static void free_job_arrays(verify_job* j) {
  free(j->job_off);
  free(j->pk_off);
  free(j->job_result);
  free(j->parts);
  j->job_off = j->pk_off = NULL;
  j->job_result = NULL;
  j->parts = NULL;
}

/* reads the batch object into j->b; copies the offsets; pins the other arrays when pin != 0 */
static int read_batch(napi_env env, napi_value obj, verify_job* j, int pin) {
  void* p[N_FIELDS] = {0};
  size_t n[N_FIELDS] = {0};
  napi_value v[N_FIELDS];
  for (int k = 0; k < N_FIELDS; k++) {
    bool has = false;
    napi_has_named_property(env, obj, FIELD[k], &has);
    if (!has) {
      if (k == F_RAW) continue;
      napi_throw_type_error(env, NULL, "batch field missing");
      return -1;
    }
    napi_get_named_property(env, obj, FIELD[k], &v[k]);
    if (typed(env, v[k], FIELD_T[k], &p[k], &n[k])) {
      napi_throw_type_error(env, NULL, "batch field has the wrong typed-array type");
      return -1;
    }
  }
  if (n[F_JOB] < 1 || n[F_PKO] < 1) {
    napi_throw_range_error(env, NULL, "jobOffsets / pkOffsets need at least one entry");
    return -1;
  }
  memset(&j->b, 0, sizeof j->b);
  j->b.n_jobs = (uint32_t)(n[F_JOB] - 1);
  j->b.n_sets = (uint32_t)(n[F_PKO] - 1);
  j->job_off = (uint32_t*)malloc(4 * n[F_JOB]);
  j->pk_off = (uint32_t*)malloc(4 * n[F_PKO]);
  if (!j->job_off || !j->pk_off) {
    napi_throw_error(env, NULL, "out of memory");
    return -1;
  }
  memcpy(j->job_off, p[F_JOB], 4 * n[F_JOB]);
  memcpy(j->pk_off, p[F_PKO], 4 * n[F_PKO]);
  const uint32_t n_sets = j->b.n_sets;
  if (n[F_MSG] < 32ull * n_sets || n[F_SIG] < 192ull * n_sets || n[F_LEN] < n_sets) {
    napi_throw_range_error(env, NULL, "msgs / sigs / sigLen shorter than the set count");
    return -1;
  }
  if (n[F_PKI] < (size_t)j->pk_off[n_sets]) {
    napi_throw_range_error(env, NULL, "pkIndices shorter than pkOffsets[n_sets]");
    return -1;
  }
  if (pin)
    for (int k = 0; k < N_FIELDS; k++)
      if (p[k] && k != F_JOB && k != F_PKO) napi_create_reference(env, v[k], 1, &j->refs[k]);
  j->b.job_offsets = j->job_off;
  j->b.pk_offsets = j->pk_off;
  j->b.pk_indices = (const uint32_t*)p[F_PKI];
  j->b.msgs = (const uint8_t*)p[F_MSG];
  j->b.sigs = (const uint8_t*)p[F_SIG];
  j->b.sig_len = (const uint32_t*)p[F_LEN];
  j->b.raw_pks = (const uint8_t*)p[F_RAW];
  j->b.n_raw = (uint32_t)(n[F_RAW] / 96);
  j->b.scalars = NULL; /* drawn inside the library (device ChaCha20 keyed by getrandom) */
  j->b.on_device = 0;
  return 0;
}

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

static void run_verify(verify_job* j) {
  pthread_mutex_lock(&j->c->mu);
  j->t_start_ms = now_ms();
  if (j->c->closed) {
    j->status = BGV_E_INVALID_ARG;
    snprintf(j->err, sizeof j->err, "QUEUE_ERROR_QUEUE_ABORTED");
  } else {
    switch (j->kind) {
      case K_PARTIAL:
        j->status = bgv_partial(j->c->ctx, &j->b, j->miller, NULL, j->job_result, &j->ok);
        j->c->partial_jobs = j->b.n_jobs;
        if (j->status == BGV_OK) {
          j->status = bgv_last_stats(j->c->ctx, &j->stats);
          j->stats.pubkeys_aggregated = j->b.n_sets ? j->pk_off[j->b.n_sets] : 0;
        }
        break;
      case K_FINISH:
        j->b.n_jobs = j->c->partial_jobs;
        j->job_result = (int32_t*)calloc(j->b.n_jobs ? j->b.n_jobs : 1, 4);
        j->status = j->job_result ? bgv_partial_finish(j->c->ctx, j->job_result, &j->stats) : BGV_E_INVALID_ARG;
        break;
      case K_COMBINE: j->status = bgv_combine_final(j->c->ctx, j->parts, j->n_parts, &j->ok); break;
      default: j->status = bgv_verify(j->c->ctx, &j->b, j->job_result, NULL, &j->stats); break;
    }
    if (j->status != BGV_OK) snprintf(j->err, sizeof j->err, "bgv error %d: %s", j->status, bgv_last_error());
  }
  j->t_end_ms = now_ms();
  pthread_mutex_unlock(&j->c->mu);
}

/* {results, batchRetries, batchSigsSuccess, pubkeysAggregated, deviceMs, workerStartMs, workerEndMs} */
static napi_value result_object(napi_env env, const verify_job* j) {
  napi_value o, v;
  if (napi_create_object(env, &o) != napi_ok) return NULL;
  v = new_int32_array(env, j->job_result, j->b.n_jobs);
  if (!v) return NULL;
  napi_set_named_property(env, o, "results", v);
  napi_create_uint32(env, j->stats.batch_retries, &v);
  napi_set_named_property(env, o, "batchRetries", v);
  napi_create_uint32(env, j->stats.batch_sigs_success, &v);
  napi_set_named_property(env, o, "batchSigsSuccess", v);
  napi_create_double(env, (double)j->stats.pubkeys_aggregated, &v);
  napi_set_named_property(env, o, "pubkeysAggregated", v);
  napi_create_double(env, (double)j->stats.total_ms, &v);
  napi_set_named_property(env, o, "deviceMs", v);
  napi_create_double(env, j->t_start_ms, &v);
  napi_set_named_property(env, o, "workerStartMs", v);
  napi_create_double(env, j->t_end_ms, &v);
  napi_set_named_property(env, o, "workerEndMs", v);
  if (j->kind == K_PARTIAL) {
    void* dst = NULL;
    napi_value ab;
    if (napi_create_arraybuffer(env, 576, &dst, &ab) != napi_ok) return NULL;
    memcpy(dst, j->miller, 576);
    napi_create_typedarray(env, napi_uint8_array, 576, ab, 0, &v);
    napi_set_named_property(env, o, "miller", v);
    napi_get_boolean(env, j->ok != 0, &v);
    napi_set_named_property(env, o, "ok", v);
  }
  return o;
}

static void exec_verify(napi_env env, void* data) { /* libuv worker thread */
  (void)env;
  run_verify((verify_job*)data);
}

static void done_verify(napi_env env, napi_status st, void* data) { /* main thread */
  verify_job* j = (verify_job*)data;
  if (st != napi_ok && j->status == BGV_OK) {
    j->status = BGV_E_INVALID_ARG;
    snprintf(j->err, sizeof j->err, "async work cancelled");
  }
  if (j->status != BGV_OK) {
    napi_value msg, err;
    napi_create_string_utf8(env, j->err, NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  } else if (j->kind == K_COMBINE) {
    napi_value b;
    napi_get_boolean(env, j->ok != 0, &b);
    napi_resolve_deferred(env, j->deferred, b);
  } else {
    napi_resolve_deferred(env, j->deferred, result_object(env, j));
  }
  for (int k = 0; k < N_FIELDS; k++)
    if (j->refs[k]) napi_delete_reference(env, j->refs[k]); /* unpin the inputs */
  if (j->ctx_ref) napi_delete_reference(env, j->ctx_ref);
  napi_delete_async_work(env, j->work);
  free_job_arrays(j);
  free(j);
}

/* queue j on the libuv pool; the promise settles in done_verify */
static napi_value queue_job(napi_env env, napi_value ctx_val, verify_job* j, const char* label) {
  napi_create_reference(env, ctx_val, 1, &j->ctx_ref); /* the context outlives its queued work */
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_CALL(env, napi_create_string_utf8(env, label, NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, exec_verify, done_verify, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  return promise;
}

static napi_value queue_batch(napi_env env, napi_callback_info info, int kind, const char* label) {
  size_t argc = 2;
  napi_value a[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  verify_job* j = (verify_job*)calloc(1, sizeof *j);
  j->c = c;
  j->kind = kind;
  if (read_batch(env, a[1], j, 1)) {
    for (int k = 0; k < N_FIELDS; k++)
      if (j->refs[k]) napi_delete_reference(env, j->refs[k]);
    free_job_arrays(j);
    free(j);
    return NULL;
  }
  j->job_result = (int32_t*)calloc(j->b.n_jobs ? j->b.n_jobs : 1, 4);
  return queue_job(env, a[0], j, label);
}

static napi_value Verify(napi_env env, napi_callback_info info) { return queue_batch(env, info, K_VERIFY, "bgv_verify"); }

static napi_value Partial(napi_env env, napi_callback_info info) { return queue_batch(env, info, K_PARTIAL, "bgv_partial"); }

/* partialFinish(ctx): the shard left by the last partial() on the context */
static napi_value PartialFinish(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value a[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  verify_job* j = (verify_job*)calloc(1, sizeof *j);
  j->c = c;
  j->kind = K_FINISH; /* results sized on the pool thread from the pending partial */
  return queue_job(env, a[0], j, "bgv_partial_finish");
}

static napi_value CombineFinal(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value a[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  void* data;
  size_t len;
  if (argc < 2 || typed(env, a[1], napi_uint8_array, &data, &len) || len % 576) {
    napi_throw_type_error(env, NULL, "combineFinal(ctx, Uint8Array of 576-byte partials)");
    return NULL;
  }
  verify_job* j = (verify_job*)calloc(1, sizeof *j);
  j->c = c;
  j->kind = K_COMBINE;
  j->n_parts = (uint32_t)(len / 576);
  j->parts = (uint8_t*)malloc(len ? len : 1); /* copied: the caller may reuse its buffer */
  if (len) memcpy(j->parts, data, len);
  return queue_job(env, a[0], j, "bgv_combine_final");
}

static napi_value VerifySync(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value a[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, a, NULL, NULL));
  addon_ctx* c = get_ctx(env, a[0]);
  if (!c) return NULL;
  verify_job j;
  memset(&j, 0, sizeof j);
  j.c = c;
  if (read_batch(env, a[1], &j, 0)) {
    free_job_arrays(&j);
    return NULL;
  }
  j.job_result = (int32_t*)calloc(j.b.n_jobs ? j.b.n_jobs : 1, 4);
  run_verify(&j);
  napi_value r = NULL;
  if (j.status != BGV_OK) napi_throw_error(env, NULL, j.err);
  else r = result_object(env, &j);
  free_job_arrays(&j);
  return r;
}

static napi_value Init(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
      {"abiVersion", NULL, AbiVersion, NULL, NULL, NULL, napi_enumerable, NULL},
      {"buildId", NULL, BuildId, NULL, NULL, NULL, napi_enumerable, NULL},
      {"codeName", NULL, CodeName, NULL, NULL, NULL, napi_enumerable, NULL},
      {"open", NULL, Open, NULL, NULL, NULL, napi_enumerable, NULL},
      {"close", NULL, Close, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pubkeysSet", NULL, PubkeysSet, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pubkeysCount", NULL, PubkeysCount, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pubkeysValidate", NULL, PubkeysValidate, NULL, NULL, NULL, napi_enumerable, NULL},
      {"verify", NULL, Verify, NULL, NULL, NULL, napi_enumerable, NULL},
      {"verifySync", NULL, VerifySync, NULL, NULL, NULL, napi_enumerable, NULL},
      {"partial", NULL, Partial, NULL, NULL, NULL, napi_enumerable, NULL},
      {"partialFinish", NULL, PartialFinish, NULL, NULL, NULL, napi_enumerable, NULL},
      {"combineFinal", NULL, CombineFinal, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  if (napi_define_properties(env, exports, sizeof d / sizeof d[0], d) != napi_ok) return NULL;
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
