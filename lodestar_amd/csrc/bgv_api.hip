// Host side of the C ABI declared in include/bgv.h: context, HBM-resident
// pubkey table, batch staging and the stage pipeline on one HIP stream.
//
// Reference behaviour re-created (packages/beacon-node/src/chain/bls/):
//   * multithread/worker.ts:30-106  one batch check, per-job fallback
//   * maybeBatch.ts:16-38           job verdict = AND of its sets; parse
//                                    errors reject the job
//   * utils.ts:5-16                 pubkey aggregation (now on the device)
//   * multithread/index.ts:193-214  close()
#include <sys/random.h>
#include <string.h>
#include <stdio.h>
#include <stdarg.h>
#include <stdlib.h>
#include <atomic>
#include <vector>
#include <string>

#include "bgv_internal.h"
#include "../../include/bgv.h"

using namespace bgv;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) return fail(BGV_E_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

template <class T>
struct dbuf {
  T* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    size_t c = cap ? cap : 64;
    while (c < n) c *= 2;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc((void**)&p, c * sizeof(T)) != hipSuccess) return fail(BGV_E_HIP, "hipMalloc(%zu) failed", c * sizeof(T));
    cap = c;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct bgv_ctx {
  int device = 0;
  bgv_cfg cfg;            // pipeline overrides (bgv_open_cfg; all "auto" from bgv_open)
  bool timed = true;      // the last run_stages recorded per-stage events
  int run_from = 0, run_to = 0;  // stage range of the last run_stages (bgv_last_stats)
  dev_batch last_d = {};         // the last run_stages batch (its pipeline variant for bgv_stats)
  hipStream_t st = nullptr, st_hash = nullptr, st_pk = nullptr;
  bool busy = false;  // prepare(): another batch of this process was in flight on the device
  hipStream_t st_chk = nullptr;  // deferred subgroup checks, low priority (BGV_CHK_STREAM)
  hipEvent_t ev[ST_COUNT + 1] = {};   // ev[s] = start of stage s on its stream
  hipEvent_t ev_end[ST_COUNT] = {};   // end of stage s on its stream
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_prep = nullptr;       // end of launch_prep (latency batches fork the hash leg before it)
  hipEvent_t ev_sigdec = nullptr;     // defer_grp: signatures decoded (the checks may start)
  hipEvent_t ev_grp = nullptr;        // defer_grp: subgroup checks done (the code fix-up may start)
  hipEvent_t ev_maps = nullptr;       // early_maps: the hash maps on st_hash are done
  hipEvent_t ev_chk = nullptr;        // pubkey scaling done: the deferred checks may start on st_chk
  hipEvent_t ev_dep[ST_COUNT] = {};   // untimed cross-stream dependencies (latency batches)
  // index2pubkey table (grown by copy) and synthetic secret keys
  g1a* table = nullptr;
  uint32_t table_n = 0, table_cap = 0;
  dbuf<uint32_t> sk;
  // staging for host batches: every host array of a batch is packed into one
  // pinned buffer and crosses PCIe in ONE copy (pageable copies cost ~30-90 us
  // each on the C2 critical path); results come back through pinned memory too
  dbuf<uint8_t> stage_dev;
  uint8_t* pin_in = nullptr;
  uint8_t* pin_out = nullptr;
  size_t pin_in_cap = 0, pin_out_cap = 0;
  hipEvent_t ev_staged = nullptr;  // the last pin_in -> stage_dev copy
  bool staged_pending = false;
  dbuf<uint8_t> raw_in, gen_out;
  dbuf<g1a> pk_tmp;         // bgv_pubkeys_set: decoded rows before they enter the table
  dbuf<int32_t> pk_codes;   // bgv_pubkeys_set: per-key deserialization codes
  std::vector<int32_t> pk_codes_host;
  // host view of the last prepared batch (offsets from the pinned copy or HBM)
  std::vector<uint32_t> jo_host;
  uint32_t pk_total = 0;
  // bgv_partial -> bgv_partial_finish: the shard's intermediates stay resident
  bool partial_pending = false;
  dev_batch part_d;
  dev_work part_w;
  // bgv_debug_stages
  dbuf<g1a> pk_agg;
  dbuf<fp12_t> dbg_fe, dbg_f;
  dbuf<uint8_t> dbg_out;
  dbuf<uint64_t> scalars;
  dbuf<g1a> raw_conv;
  // per-batch intermediates
  dbuf<g2a> sig_aff, h_aff;
  dbuf<uint32_t> sig_inf, flags;
  dbuf<int32_t> sig_code, pk_code, job_code, job_result, set_code;
  dbuf<g1a> rpk_aff;
  dbuf<uint32_t> chunk_off, chunk_set;
  dbuf<g1j> pk_part;
  dbuf<g2j> rsig, q_part;
  dbuf<uint32_t> sig_grp;
  dbuf<fp2_t> lines;
  uint32_t lines_idle = 0;  // batches in a row that did not use the line buffer
  dbuf<fp12_t> f_set, f_job, f_batch, f_tmp, f_part;
  dbuf<uint32_t> set_job, s_inf, item_off, item_job;
  dbuf<g2a> s_aff;
  dbuf<g2j> msm_bucket, msm_win;
  dbuf<uint32_t> msm_mask;
  // microbench scratch
  dbuf<fp_t> mb_fp;
  dbuf<uint64_t> mb_u64;
};

// Definitions below take C linkage from their declarations in bgv.h.

int bgv_abi_version(void) { return BGV_ABI_VERSION; }
#ifndef BGV_SRC_HASH
#define BGV_SRC_HASH "unhashed"
#endif
const char* bgv_build_id(void) { return BGV_SRC_HASH; }
const char* bgv_last_error(void) { return g_err.c_str(); }

const char* bgv_set_code_name(int code) {
  switch (code) {
    case 0: return "BLST_SUCCESS";
    case 1: return "BLST_BAD_ENCODING";
    case 2: return "BLST_POINT_NOT_ON_CURVE";
    case 3: return "BLST_POINT_NOT_IN_GROUP";
    case 4: return "BLST_AGGR_TYPE_MISMATCH";
    case 5: return "BLST_VERIFY_FAIL";
    case 6: return "BLST_PK_IS_INFINITY";
    case 7: return "BLST_BAD_SCALAR";
    case 8: return "BLST_INVALID_SIZE";
    case 9: return "BGV_INDEX_RANGE";
    case 10: return "EMPTY_SIGNATURE_SET";
    default: return "BGV_UNKNOWN";
  }
}

const char* bgv_stage_name(int stage) {
  static const char* names[ST_COUNT] = {"sig_decode_subgroup", "hash_to_g2",       "pk_gather",
                                        "pk_aggregate_scale",  "sig_scale",        "sig_sum_tree",
                                        "miller_loop",         "miller_loop_jobs", "miller_product_tree",
                                        "batch_product",       "batch_final_exp",  "job_final_exp",
                                        "set_codes"};
  return (stage >= 0 && stage < ST_COUNT) ? names[stage] : "unknown";
}

void bgv_cfg_default(bgv_cfg* cfg) {
  if (!cfg) return;
  memset(cfg, 0, sizeof *cfg);
  cfg->struct_size = sizeof *cfg;
  cfg->split = cfg->miller = cfg->msm = cfg->prefold = cfg->lines = cfg->defer_pct = cfg->timing = cfg->clear_lanes = -1;
  cfg->miller_kv = -1;
  cfg->job_lanes = cfg->pairs = cfg->cu_split = 0;
}

int bgv_open(int device, bgv_ctx** out) { return bgv_open_cfg(device, nullptr, out); }

int bgv_open_cfg(int device, const bgv_cfg* cfg, bgv_ctx** out) {
  if (!out) return fail(BGV_E_INVALID_ARG, "out is NULL");
  *out = nullptr;
  bgv_cfg k;
  bgv_cfg_default(&k);
  if (cfg) {
    if (cfg->struct_size != sizeof k) return fail(BGV_E_INVALID_ARG, "bgv_cfg.struct_size %u, expected %zu", cfg->struct_size, sizeof k);
    k = *cfg;
    auto lanes_ok = [](int v) { return v == 6 || v == 18 || v == 36; };
    if (k.miller != -1 && k.miller != 1 && k.miller != 2 && k.miller != 4 && !lanes_ok(k.miller)) return fail(BGV_E_INVALID_ARG, "bgv_cfg.miller %d", k.miller);
    if (k.job_lanes != 0 && !lanes_ok(k.job_lanes)) return fail(BGV_E_INVALID_ARG, "bgv_cfg.job_lanes %d", k.job_lanes);
    if (k.pairs < 0 || k.pairs == 3 || k.pairs > 4) return fail(BGV_E_INVALID_ARG, "bgv_cfg.pairs %d", k.pairs);
    if (k.msm < -1 || k.msm > 4) return fail(BGV_E_INVALID_ARG, "bgv_cfg.msm %d", k.msm);
    if (k.clear_lanes != -1 && k.clear_lanes != 1 && k.clear_lanes != 3 && k.clear_lanes != 9)
      return fail(BGV_E_INVALID_ARG, "bgv_cfg.clear_lanes %d", k.clear_lanes);
    if (k.miller_kv != -1 && k.miller_kv != 0 && k.miller_kv != 2 && k.miller_kv != 3 && k.miller_kv != 6 && k.miller_kv != 9)
      return fail(BGV_E_INVALID_ARG, "bgv_cfg.miller_kv %d", k.miller_kv);
    if (k.defer_pct < -1 || k.defer_pct > 100) return fail(BGV_E_INVALID_ARG, "bgv_cfg.defer_pct %d", k.defer_pct);
    auto tri_ok = [](int v) { return v >= -1 && v <= 1; };
    if (!tri_ok(k.split)) return fail(BGV_E_INVALID_ARG, "bgv_cfg.split %d", k.split);
    if (!tri_ok(k.prefold)) return fail(BGV_E_INVALID_ARG, "bgv_cfg.prefold %d", k.prefold);
    if (!tri_ok(k.lines)) return fail(BGV_E_INVALID_ARG, "bgv_cfg.lines %d", k.lines);
    if (!tri_ok(k.timing)) return fail(BGV_E_INVALID_ARG, "bgv_cfg.timing %d", k.timing);
    if (k.cu_split < -64 || k.cu_split > 64) return fail(BGV_E_INVALID_ARG, "bgv_cfg.cu_split %d (|N| <= 64 CUs)", k.cu_split);
    // two pairs per item exist only in the one-lane loop
    if (k.pairs >= 2 && k.miller != -1 && k.miller != 1)
      return fail(BGV_E_INVALID_ARG, "bgv_cfg.pairs 2 needs the one-lane Miller loop (miller %d)", k.miller);
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(BGV_E_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(BGV_E_NO_DEVICE, "device %d out of range (%d devices)", device, n);
  HIPCHK(hipSetDevice(device));
  // CU partition between a priority context (the |N| highest CU ids) and the
  // bulk contexts (the rest): a single set's few waves then never queue
  // behind a resident bulk batch (k_hash alone holds two waves on every SIMD
  // for ~16 ms at C4).  Streams with a CU mask take no priority.  Mask bit i
  // is CU i / 8 of XCC i % 8, in shader engine (i / 8) % 4
  // (tools/cu_mask_probe.hip, probed on MI355X: 8 XCCs x 32 CUs), and an XCC
  // left without any bit runs on all of its CUs, so N must be a multiple of
  // the XCC count: the highest 8k ids then take k CUs from every XCC (32: one
  // per SE).  Any other layout is refused rather than half-isolated.
  // Workgroups go round-robin over the SEs, so the bulk side runs at the pace
  // of an SE that lost a CU: C4 +13% for 8, 16 or 32 reserved CUs alike
  // (profiles/r05h_cu_split.txt).
  std::vector<uint32_t> mask;
  if (k.cu_split != 0) {
    int n_cu = 0, n_xcc = 0;
    HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
    if (hipDeviceGetAttribute(&n_xcc, hipDeviceAttributeNumberOfXccs, device) != hipSuccess) n_xcc = 0;
    const int reserve = k.cu_split > 0 ? k.cu_split : -k.cu_split;
    if (n_xcc != 8 || n_cu != 256)
      return fail(BGV_E_INVALID_ARG, "bgv_cfg.cu_split %d: the CU-mask layout is probed for 8 XCCs x 32 CUs (device: %d XCCs, %d CUs)",
                  k.cu_split, n_xcc, n_cu);
    if (reserve % n_xcc != 0)
      return fail(BGV_E_INVALID_ARG, "bgv_cfg.cu_split %d: |N| must be a multiple of the %d XCCs (an XCC without a mask bit runs on all its CUs)",
                  k.cu_split, n_xcc);
    mask.assign((size_t)(n_cu + 31) / 32, 0u);
    for (int cu = 0; cu < n_cu; cu++) {
      const bool reserved = cu >= n_cu - reserve;
      if (reserved == (k.cu_split > 0)) mask[cu / 32] |= 1u << (cu % 32);
    }
  }
  bgv_ctx* c = new bgv_ctx();
  c->device = device;
  c->cfg = k;
  // on a failure below, the streams and events made so far go with the context
  struct guard_t {
    bgv_ctx*& c;
    ~guard_t() { if (c) bgv_close(c); }
  } guard{c};
  // hash -> set-pair Miller is the critical path: its stream (and the pubkey
  // stream feeding it) get the highest priority, signature decode/scaling the
  // lowest (it only feeds the signature tree and the 1 pair per job)
  int prio_lo = 0, prio_hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  if (k.cu_split == 0) {
    HIPCHK(hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, prio_lo));
    HIPCHK(hipStreamCreateWithPriority(&c->st_hash, hipStreamNonBlocking, prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&c->st_pk, hipStreamNonBlocking, prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&c->st_chk, hipStreamNonBlocking, prio_lo));
  } else {
    hipStream_t* sts[4] = {&c->st, &c->st_hash, &c->st_pk, &c->st_chk};
    for (hipStream_t* p : sts) HIPCHK(hipExtStreamCreateWithCUMask(p, (uint32_t)mask.size(), mask.data()));
  }
  for (auto& e : c->ev) HIPCHK(hipEventCreate(&e));
  for (auto& e : c->ev_end) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventCreate(&c->ev_fork));
  HIPCHK(hipEventCreateWithFlags(&c->ev_staged, hipEventDisableTiming));
  for (auto& e : c->ev_dep) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&c->ev_prep, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&c->ev_sigdec, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&c->ev_grp, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&c->ev_maps, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&c->ev_chk, hipEventDisableTiming));
  *out = c;
  c = nullptr;  // owned by the caller now
  return BGV_OK;
}

int bgv_close(bgv_ctx* c) {
  if (!c) return BGV_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->st);
  (void)hipStreamSynchronize(c->st_hash);
  (void)hipStreamSynchronize(c->st_pk);
  (void)hipStreamSynchronize(c->st_chk);
  for (auto& e : c->ev) (void)hipEventDestroy(e);
  for (auto& e : c->ev_end) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->ev_fork);
  (void)hipEventDestroy(c->ev_staged);
  for (auto& e : c->ev_dep) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->ev_prep);
  (void)hipEventDestroy(c->ev_sigdec);
  (void)hipEventDestroy(c->ev_grp);
  (void)hipEventDestroy(c->ev_maps);
  (void)hipEventDestroy(c->ev_chk);
  if (c->pin_in) (void)hipHostFree(c->pin_in);
  if (c->pin_out) (void)hipHostFree(c->pin_out);
  if (c->table) (void)hipFree(c->table);
  c->sk.release();
  c->stage_dev.release();
  c->raw_in.release(); c->gen_out.release(); c->pk_tmp.release(); c->pk_codes.release();
  c->pk_agg.release(); c->dbg_fe.release(); c->dbg_f.release(); c->dbg_out.release();
  c->scalars.release(); c->raw_conv.release();
  c->sig_aff.release(); c->h_aff.release(); c->sig_inf.release(); c->flags.release();
  c->sig_code.release(); c->pk_code.release(); c->job_code.release(); c->job_result.release(); c->set_code.release();
  c->rpk_aff.release(); c->chunk_off.release(); c->chunk_set.release(); c->pk_part.release(); c->rsig.release(); c->q_part.release(); c->sig_grp.release(); c->lines.release(); c->f_set.release(); c->f_job.release(); c->f_batch.release(); c->f_tmp.release(); c->f_part.release();
  c->msm_bucket.release(); c->msm_win.release(); c->msm_mask.release();
  c->set_job.release(); c->s_inf.release(); c->item_off.release(); c->item_job.release(); c->s_aff.release();
  c->mb_fp.release(); c->mb_u64.release();
  (void)hipStreamDestroy(c->st);
  (void)hipStreamDestroy(c->st_hash);
  (void)hipStreamDestroy(c->st_pk);
  (void)hipStreamDestroy(c->st_chk);
  delete c;
  return BGV_OK;
}

static int table_reserve(bgv_ctx* c, uint32_t n) {
  if (n <= c->table_cap) return 0;
  uint32_t cap = c->table_cap ? c->table_cap : 1024;
  while (cap < n) cap = cap * 2u > cap ? cap * 2u : n;
  g1a* t = nullptr;
  HIPCHK(hipMalloc((void**)&t, (size_t)cap * sizeof(g1a)));
  HIPCHK(hipMemsetAsync(t, 0, (size_t)cap * sizeof(g1a), c->st));
  if (c->table) {
    HIPCHK(hipMemcpyAsync(t, c->table, (size_t)c->table_n * sizeof(g1a), hipMemcpyDeviceToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    HIPCHK(hipFree(c->table));
  }
  c->table = t;
  c->table_cap = cap;
  return 0;
}

// index2pubkey rows are u32 indices with bit 31 reserved for raw_pks
static const uint32_t TABLE_MAX = 0x7fffffffu;

int bgv_pubkeys_set(bgv_ctx* c, uint32_t first, uint32_t n, const uint8_t* data, uint32_t fmt) {
  if (!c || (!data && n)) return fail(BGV_E_INVALID_ARG, "null argument");
  if (fmt != BGV_PK_COMPRESSED_48 && fmt != BGV_PK_UNCOMPRESSED_96) return fail(BGV_E_INVALID_ARG, "bad format %u", fmt);
  c->partial_pending = false;
  if (n == 0) return BGV_OK;
  if ((uint64_t)first + n > TABLE_MAX) return fail(BGV_E_TABLE_RANGE, "rows [%u, %llu) exceed the table limit 2^31 - 1", first, (unsigned long long)first + n);
  if (first > c->table_n)
    return fail(BGV_E_TABLE_RANGE, "row %u would leave a gap after the %u rows of the table (append-only, pubkeyCache.ts:56-77)", first, c->table_n);
  HIPCHK(hipSetDevice(c->device));
  if (int r = table_reserve(c, first + n)) return r;
  const size_t w = fmt == BGV_PK_COMPRESSED_48 ? 48 : 96;
  if (int r = c->raw_in.ensure((size_t)n * w)) return r;
  if (int r = c->pk_tmp.ensure(n)) return r;
  if (int r = c->pk_codes.ensure(n)) return r;
  HIPCHK(hipMemcpyAsync(c->raw_in.p, data, (size_t)n * w, hipMemcpyHostToDevice, c->st));
  if (fmt == BGV_PK_COMPRESSED_48) launch_table_from_compressed(c->st, c->raw_in.p, c->pk_tmp.p, n, c->pk_codes.p);
  else launch_table_from_uncompressed(c->st, c->raw_in.p, c->pk_tmp.p, n, c->pk_codes.p);
  HIPCHK(hipGetLastError());
  c->pk_codes_host.resize(n);
  HIPCHK(hipMemcpyAsync(c->pk_codes_host.data(), c->pk_codes.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  for (uint32_t i = 0; i < n; i++)
    if (c->pk_codes_host[i] != 0)  // PublicKey.fromBytes throws: nothing is stored
      return fail(BGV_E_BAD_PUBKEY, "pubkey %u: BLST_ERROR: %s", first + i, bgv_set_code_name(c->pk_codes_host[i]));
  HIPCHK(hipMemcpyAsync(c->table + first, c->pk_tmp.p, (size_t)n * sizeof(g1a), hipMemcpyDeviceToDevice, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  if (first + n > c->table_n) c->table_n = first + n;
  return BGV_OK;
}

int bgv_pubkeys_count(bgv_ctx* c, uint32_t* count) {
  if (!c || !count) return fail(BGV_E_INVALID_ARG, "null argument");
  *count = c->table_n;
  return BGV_OK;
}

int bgv_pubkeys_get(bgv_ctx* c, uint32_t first, uint32_t n, uint8_t* out96) {
  if (!c || (!out96 && n)) return fail(BGV_E_INVALID_ARG, "null argument");
  if ((uint64_t)first + n > c->table_n) return fail(BGV_E_TABLE_RANGE, "range [%u, %u) beyond table size %u", first, first + n, c->table_n);
  if (n == 0) return BGV_OK;
  HIPCHK(hipSetDevice(c->device));
  if (int r = c->gen_out.ensure((size_t)n * 96)) return r;
  launch_table_export(c->st, c->table + first, c->gen_out.p, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out96, c->gen_out.p, (size_t)n * 96, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return BGV_OK;
}

int bgv_pubkeys_validate(bgv_ctx* c, const uint8_t* pk48, uint32_t n, int32_t* codes) {
  if (!c || (n && (!pk48 || !codes))) return fail(BGV_E_INVALID_ARG, "null argument");
  if (n == 0) return BGV_OK;
  HIPCHK(hipSetDevice(c->device));
  if (int r = c->raw_in.ensure((size_t)n * 48)) return r;
  if (int r = c->sig_code.ensure(n)) return r;
  HIPCHK(hipMemcpyAsync(c->raw_in.p, pk48, (size_t)n * 48, hipMemcpyHostToDevice, c->st));
  launch_pk_validate(c->st, c->raw_in.p, n, c->sig_code.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(codes, c->sig_code.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return BGV_OK;
}

// ---------------------------------------------------------------- batches

static void random_bytes(void* out, size_t n) {
  size_t got = 0;
  uint8_t* p = (uint8_t*)out;
  while (got < n) {
    ssize_t r = getrandom(p + got, n - got, 0);
    if (r > 0) got += (size_t)r;
  }
}

// a device allocation of prepare(): under memory pressure a kept line buffer
// (up to 2.6 GB, see work_alloc) gives way first, then the allocation retries
template <class T>
static int ensure_or_release_lines(bgv_ctx* c, dbuf<T>& b, size_t n) {
  int r = b.ensure(n);
  if (r && c->lines.cap && (const void*)&b != (const void*)&c->lines) {
    c->lines.release();
    c->lines_idle = 0;
    r = b.ensure(n);
  }
  return r;
}

static int pinned_reserve(uint8_t*& p, size_t& cap, size_t n) {
  if (n <= cap) return 0;
  size_t c = cap ? cap : 65536;
  while (c < n) c *= 2;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  if (hipHostMalloc((void**)&p, c, hipHostMallocDefault) != hipSuccess) return fail(BGV_E_HIP, "hipHostMalloc(%zu) failed", c);
  cap = c;
  return 0;
}

// one host array of a batch, packed at a 256-byte aligned offset of the staging buffers
struct stage_seg {
  const void* src;
  size_t bytes;
  const void** dst;
  size_t off;  // filled by stage_pack: offset in pin_in / stage_dev
};

// pack the segments into pin_in (host copies only) and point every *dst at
// its future device copy; stage_issue then moves the whole buffer in one transfer
static int stage_pack(bgv_ctx* c, stage_seg* segs, int n_segs, size_t& total) {
  total = 0;
  for (int i = 0; i < n_segs; i++) total += (segs[i].bytes + 255) & ~size_t(255);
  if (c->staged_pending) {  // the previous batch's copy may still read pin_in
    HIPCHK(hipEventSynchronize(c->ev_staged));
    c->staged_pending = false;
  }
  if (int r = pinned_reserve(c->pin_in, c->pin_in_cap, total ? total : 1)) return r;
  if (int r = ensure_or_release_lines(c, c->stage_dev, total ? total : 1)) return r;
  size_t off = 0;
  for (int i = 0; i < n_segs; i++) {
    if (segs[i].bytes) memcpy(c->pin_in + off, segs[i].src, segs[i].bytes);
    segs[i].off = off;
    *segs[i].dst = c->stage_dev.p + off;
    off += (segs[i].bytes + 255) & ~size_t(255);
  }
  return 0;
}

static int stage_issue(bgv_ctx* c, size_t total) {
  if (!total) return 0;
  HIPCHK(hipMemcpyAsync(c->stage_dev.p, c->pin_in, total, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipEventRecord(c->ev_staged, c->st));
  c->staged_pending = true;
  return 0;
}

// latency mode by batch size (prepare(); the r02 sweep: 25,088 sets 24.5 ms
// split against 26.3 ms, 50,176: 35.4 against 29.3; r03: to 65,536)
static const uint32_t SPLIT_MAX = 59000;
// With other batches in flight on the device (this process's bgv_verify /
// bgv_partial calls between entry and results), batches from INFLIGHT_BULK_MIN
// sets take the bulk pipeline (one lane per set, two pairs per Miller item over
// lines), whose kernels do the most work per instruction: with three in flight
// 50,176 sets 19.7-19.8 -> 18.5-18.8 ms per batch, 37,632 sets 15.8-16.4 ->
// 14.8-15.1 (profiles/r06ag_c4_over_2/); alone it loses (23.3-23.8 -> 29.1-29.8).
static const uint32_t INFLIGHT_BULK_MIN = 32000;
static std::atomic<int> g_active[64];
struct active_guard {
  int dev;
  explicit active_guard(int d) : dev(d >= 0 && d < 64 ? d : -1) { if (dev >= 0) g_active[dev]++; }
  ~active_guard() { if (dev >= 0) g_active[dev]--; }
};
static bool layout_split(const bgv_cfg& k, uint32_t n, bool busy) {
  return k.split >= 0 ? k.split != 0 : (n < SPLIT_MAX && !(busy && n >= INFLIGHT_BULK_MIN));
}

// The hash maps of a latency-mode batch read only the messages, and they head
// the critical path (maps -> clearing -> Miller -> fold -> final exp): they are
// launched on the hash stream as soon as the messages are on the device,
// before the host reads back offsets, checks them and sets up the rest
// (on-device batches: ~0.1 ms of idle GPU at 3,136 sets, r04c timeline).
// Timed runs keep the maps inside the hash stage's events.
#ifndef BGV_CHK_STREAM
#define BGV_CHK_STREAM 1
#endif
#ifndef BGV_EARLY_MAPS
#define BGV_EARLY_MAPS 1
#endif
static int early_maps(bgv_ctx* c, dev_batch& d, bool after_staging) {
  const uint32_t n = d.n_sets;
  if (!BGV_EARLY_MAPS) return 0;
  const bool timed = c->cfg.timing >= 0 ? c->cfg.timing != 0 : n >= 65536;
  if (!n || timed || !layout_split(c->cfg, n, c->busy)) return 0;
  if (int r = ensure_or_release_lines(c, c->q_part, 2 * (size_t)n)) return r;
  if (after_staging) HIPCHK(hipStreamWaitEvent(c->st_hash, c->ev_staged, 0));
  dev_work w;
  memset(&w, 0, sizeof w);
  w.q_part = c->q_part.p;
  // the batch's start event goes in front of the maps (they head the critical
  // path), so stats total_ms covers them; run_stages then does not re-record it
  HIPCHK(hipEventRecord(c->ev[0], c->st_hash));
  launch_hash_maps(c->st_hash, d, w);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev_maps, c->st_hash));
  d.maps_early = 1;
  return 0;
}

// Build the device view of a batch: stage host arrays, convert raw pubkeys.
// Host batches: the arrays are copied into pinned memory FIRST and every
// contract check reads that copy, so the device only ever sees checked
// offsets even if the caller's buffers change during the call.  Index ranges
// are checked per set on the device (BGV_SET_INDEX_RANGE rejects the job).
static int prepare(bgv_ctx* c, const bgv_batch* b, dev_batch& d, bool need_sigs) {
  if (!b) return fail(BGV_E_INVALID_ARG, "batch is NULL");
  if (!b->job_offsets || !b->pk_offsets || !b->pk_indices || !b->msgs || (need_sigs && (!b->sigs || !b->sig_len)))
    return fail(BGV_E_INVALID_ARG, "missing batch array");
  if (b->n_raw && !b->raw_pks) return fail(BGV_E_INVALID_ARG, "n_raw > 0 but raw_pks is NULL");
  const uint32_t n = b->n_sets, J = b->n_jobs;
  memset(&d, 0, sizeof d);
  // another batch of this process in flight on the device (read once per batch)
  c->busy = c->device >= 0 && c->device < 64 && g_active[c->device].load() >= 2;
  d.n_sets = n;
  d.n_jobs = J;
  d.n_raw = b->n_raw;
  d.table_n = c->table_n;
  d.table = c->table;
  d.span_log2 = 7;  // device batches: trees cover jobs of <= 128 sets (multithread/index.ts:39)
  c->jo_host.resize((size_t)J + 1);
  if (!b->on_device) {
    const uint32_t total = b->pk_offsets[n];  // sizes the pk_indices copy; re-checked on the copy
    const uint8_t* raw_dev = nullptr;
    stage_seg segs[8] = {
        {b->job_offsets, ((size_t)J + 1) * 4, (const void**)&d.job_off, 0},
        {b->pk_offsets, ((size_t)n + 1) * 4, (const void**)&d.pk_off, 0},
        {b->pk_indices, (size_t)total * 4, (const void**)&d.pk_idx, 0},
        {b->msgs, (size_t)n * 32, (const void**)&d.msgs, 0},
        {b->raw_pks, (size_t)b->n_raw * 96, (const void**)&raw_dev, 0},
        {b->scalars, b->scalars ? (size_t)n * 8 : 0, (const void**)&d.scalars, 0},
        {b->sigs, need_sigs ? (size_t)n * 192 : 0, (const void**)&d.sigs, 0},
        {b->sig_len, need_sigs ? (size_t)n * 4 : 0, (const void**)&d.sig_len, 0},
    };
    size_t bytes = 0;
    if (int r = stage_pack(c, segs, 8, bytes)) return r;
    const uint32_t* jo = (const uint32_t*)(c->pin_in + segs[0].off);
    const uint32_t* po = (const uint32_t*)(c->pin_in + segs[1].off);
    // host-side contract checks on the pinned copy (the reference rejects these synchronously)
    if (jo[0] != 0 || jo[J] != n) return fail(BGV_E_INVALID_ARG, "job_offsets must span [0, n_sets]");
    uint32_t max_job = 1;
    for (uint32_t j = 0; j < J; j++) {
      if (jo[j + 1] < jo[j]) return fail(BGV_E_INVALID_ARG, "job_offsets not monotone");
      if (jo[j + 1] - jo[j] > max_job) max_job = jo[j + 1] - jo[j];
    }
    d.span_log2 = 0;
    while ((1u << d.span_log2) < max_job && d.span_log2 < 16) d.span_log2++;
    if (po[0] != 0) return fail(BGV_E_INVALID_ARG, "pk_offsets[0] != 0");
    if (po[n] != total) return fail(BGV_E_INVALID_ARG, "pk_offsets changed during the call");
    for (uint32_t i = 0; i < n; i++) {
      if (po[i + 1] < po[i]) return fail(BGV_E_INVALID_ARG, "pk_offsets not monotone");
      if (po[i + 1] == po[i]) return fail(BGV_E_EMPTY_SET, "EMPTY_AGGREGATE_ARRAY (set %u)", i);
    }
    memcpy(c->jo_host.data(), jo, c->jo_host.size() * 4);
    c->pk_total = total;
    if (int r = stage_issue(c, bytes)) return r;
    if (need_sigs)  // verification calls (bgv_gen_sign hashes on its own)
      if (int r = early_maps(c, d, true)) return r;
    if (!b->scalars) d.scalars = nullptr;
    if (!need_sigs) { d.sigs = nullptr; d.sig_len = nullptr; }
    if (int r = ensure_or_release_lines(c, c->raw_conv, b->n_raw ? b->n_raw : 1)) return r;
    launch_raw_pks(c->st, raw_dev, c->raw_conv.p, b->n_raw);
    d.raw_pks = c->raw_conv.p;
  } else {
    d.job_off = b->job_offsets;
    d.pk_off = b->pk_offsets;
    d.pk_idx = b->pk_indices;
    d.msgs = b->msgs;
    d.sigs = b->sigs;
    d.sig_len = b->sig_len;
    if (need_sigs)
      if (int r = early_maps(c, d, false)) return r;
    if (int r = ensure_or_release_lines(c, c->raw_conv, b->n_raw ? b->n_raw : 1)) return r;
    launch_raw_pks(c->st, b->raw_pks, c->raw_conv.p, b->n_raw);
    d.raw_pks = c->raw_conv.p;
    // offsets live in HBM: the host needs the job offsets (stats) and the key total (grid bound)
    HIPCHK(hipMemcpyAsync(c->jo_host.data(), b->job_offsets, c->jo_host.size() * 4, hipMemcpyDeviceToHost, c->st));
    c->pk_total = 0;
    if (n) HIPCHK(hipMemcpyAsync(&c->pk_total, b->pk_offsets + n, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
  }
  const uint32_t total = c->pk_total;
  // grid bound of the chunked pubkey gather: sum ceil(k_i/32) <= total/32 + n
  d.chunk_bound = total / 32 + n;
  // Pipeline variant by batch size, from the r02 sweep of on-device C4-shaped
  // batches (tools/sweep_modes.py):
  //  * cooperative Miller loop (36 lanes per pair) below MILLER_COOP_MAX sets;
  //    above it the one-lane loop (36x fewer lanes) wins: 7,840 sets 20.1 ->
  //    18.2 ms, 12,544 sets 28.6 -> 20.0 ms, 50,176 sets 95.6 -> 29.3 ms;
  //  * per-job bucket MSM for sum r_i sigma_i from the same size (its 16
  //    lanes per job lengthen small batches: 98 sets 7.1 -> 17 ms);
  //  * latency mode (two-lane hash maps, cooperative G2) below SPLIT_MAX
  //    (25,088 sets: 24.5 ms split against 26.3 ms; 50,176: 35.4 against 29.3);
  //  * two pairs per Miller work item only when the batch alone fills the chip.
  //  * r03 mid-size sweep (profiles/r03_sweep_mid_sizes.jsonl): the
  //    four-lane Miller loop from 6,000 sets and the two-lane one from
  //    18,000; the three-lane cofactor clearing from 9,000; sum r_i sigma_i
  //    by the (job, window, digit)-lane MSM from 9,000 (bulk batches: the
  //    (job, window) one)
  //    (12,544: 18.4 -> 10.6 ms; 25,088: 24.1 -> 16.9 ms; 6,272: 10.8 -> 9.2 ms);
  //    the latency-mode hash (two-lane maps, one-lane clearing) with the
  //    one-lane Miller loop and the (job, window) MSM up to 65,536 sets
  //    (37,632: 25.1 -> 22.5 ms; 50,176: 26.0 -> 24.9 ms)
  //  * r04 sweeps: the one-lane Miller loop and the (job, window) MSM from
  //    32,000 sets (32,928 / 34,496 sets 25.1 / 25.3 -> 22.0 / 22.1 ms), the
  //    bulk kernels from 59,000 (62,720 sets 32.1 -> 30.3 ms, 59,584 sets
  //    30.5 -> 28.0 ms; 58,016 sets stay split: 27.1 against 28.7 ms;
  //    profiles/r04z_sweep_big.txt, profiles/r04z_sweep_split_edge.txt)
  static const uint32_t MILLER18_MIN = 2000, MILLER4_MIN = 6000, MILLER2_MIN = 15000, MILLER1_MIN = 32000, CLEAR1_MIN = 16500,
                        MSM_MIN = 6000, MSM4_MIN = 9000, MSM2_MIN = 32000, PAIRS2_MIN = 65536,
                        CLEAR3_MIN = 9000, KV6_MIN = 1100, KV3_MIN = 4500, KV_MAX = 11500;
  const bgv_cfg& k = c->cfg;
  d.pairs_per_item = k.pairs ? (uint32_t)k.pairs : (n >= PAIRS2_MIN || (c->busy && n >= INFLIGHT_BULK_MIN) ? 2u : 1u);
  d.split = layout_split(k, n, c->busy) ? 1u : 0u;
  // one lane per point from 16,500 sets (25,088: 16.74 -> 16.5 ms; 17,248:
  // 14.24 -> 13.95 ms; the trio's waves oversubscribe the SIMDs there) and the
  // two-lane Miller loop from 15,000 (r04 sweep, profiles/r04z_sweep_cliff.txt:
  // the four-lane loop's waves oversubscribe from ~15,000 sets: 15,680 sets
  // 12.38 -> 12.10 ms, 17,248 sets 16.61 -> 13.95 ms)
  d.clear_lanes = k.clear_lanes > 0 ? (uint32_t)k.clear_lanes : (n < CLEAR3_MIN ? 9u : n < CLEAR1_MIN ? 3u : 1u);
  // sum r_i sigma_i per job by a bucket MSM (16 x 4-bit windows) when jobs
  // are block-sized (<= 256 sets).  The latency mode takes the fused kernel
  // (one workgroup per job, k_msm_fused: short chain, many idle lanes); bulk
  // batches the (job, window)-lane kernels, which do a third of its SIMD-time
  // (C4: k_msm_fused 49 ms beside the hash, pubkeys and Miller loops,
  // stretching the Miller kernel from 14.5 to 26.4 ms, r03 trace)
  {
    uint32_t auto_msm = 0;
    if (n >= MSM_MIN && d.span_log2 <= 8) {
      if (!d.split || n >= MSM2_MIN) auto_msm = 2;
      else auto_msm = n < MSM4_MIN ? 1 : 4;
    }
    d.msm = k.msm >= 0 ? (uint32_t)k.msm : auto_msm;
  }
  // Deferred subgroup checks: the signature stage only decodes, and the checks
  // of sets [defer_from, n) run beside the Miller loops (bgv_kernels.hip
  // k_job_recode).  Wherever the MSM sums the signatures (the latency mode
  // without it checks beside the per-set scaling, k_sig_split_coop): all of
  // them with one pair per Miller item (C4/2 28.3 -> 26.4 ms); half with two
  // pairs per item: the Miller kernel leaves 240 SIMDs to the MSM tail and
  // the job pairs, and half of the checks fill them without outlasting it
  // (C4, 3 runs each: none 39.75, 50% 39.27, 65% 39.31, all 39.89 ms; r03, with
  // the inlined Fp12 layer: 50% 39.04 / 38.93, 75% 38.54 / 38.79, 25% 39.28 / 38.97).
  // defer_from is a multiple of 64 (wave-uniform).
  const bool deferrable = !d.split || d.msm;
  const int pct = !deferrable ? 0 : (k.defer_pct >= 0 ? k.defer_pct : (!d.split && d.pairs_per_item >= 2 ? 75 : 100));
  d.defer_grp = pct > 0 ? 1u : 0u;
  d.defer_from = pct > 0 ? (uint32_t)(((uint64_t)n * (uint32_t)(100 - pct) / 100u) & ~63ull) : n;
  // two-level per-job fold (bgv_tail.hip) for jobs of >= 64 sets: the fold
  // runs after the Miller kernels with the chip otherwise idle, so groups of
  // ~sqrt(span) sets fold side by side, then the job folds the group values,
  // 2 sqrt(span) sequential Fp12 products instead of span (r05: also for many
  // jobs; C4 product-tree stage 0.36 -> 0.33 ms, profiles/r05l_job_fold.txt)
  {
    const bool few_big = d.span_log2 >= 6 && d.span_log2 <= 8;
    const bool on = k.prefold >= 0 ? (k.prefold && d.span_log2 >= 2 && d.span_log2 <= 8) : few_big;
    d.prefold_log2 = on ? (d.span_log2 + 1) / 2 : 0u;
  }
  // set-pair Miller layout: lanes per pair shrink as the batch grows, so the
  // waves stay near one per SIMD (a pair's loop is a chain of ~1,800 Fp2
  // products on 6 lanes, ~560 product rounds on 36)
  d.miller_coop = k.miller >= 0 ? (k.miller == 1 ? 0u : (uint32_t)k.miller)
                                : (n < MILLER18_MIN ? 36u : n < MILLER4_MIN ? 18u : n < MILLER2_MIN ? 4u
                                   : n < MILLER1_MIN ? 2u : 0u);
  // two-pair Miller loop in Karatsuba views (miller_kv.h) in the latency mode:
  // the squaring of f is shared by two pairs, 3 S lanes per two pairs
  {
    // r04 sweeps (profiles/r04_sweep_kv.txt, r04c_sweep_kv_bounds.txt): 1,960
    // sets 7.57 -> 6.42 ms and 3,136 sets 6.68 -> 6.57 ms with 18 lanes per two
    // pairs (980 sets: 6.02 -> 6.18, 1,176 sets 6.70 -> 6.20: from 1,100); 4,704 sets 7.98 ->
    // 7.87, 6,272 sets 8.88 -> 8.48 ms and 10,976 sets 9.38 -> 9.17 ms with 9;
    // at 12,544 the four-lane one-pair loop stays (9.7 against 10.8 ms: the
    // 9-lane groups' 915 waves leave no SIMD to the checks and the signature chain).
    // 27 lanes per two pairs (miller_kv = 9) ties 18 at 980-1,960 sets and loses
    // from 3,136 (7.05 against 6.52 ms; profiles/r04e_sweep_kv9.txt): A/B only
    const uint32_t auto_kv = n >= KV6_MIN && n < KV3_MIN ? 6u : (n >= KV3_MIN && n < KV_MAX ? 3u : 0u);
    d.miller_kv = k.miller_kv >= 0 ? (uint32_t)k.miller_kv : auto_kv;
    if (!d.split) d.miller_kv = 0;
    if (d.miller_kv) d.pairs_per_item = 2;
    // the cooperative, four- and two-lane loops hold one pair per item (every
    // set has its own Miller value, which the per-job fold relies on)
    else if (d.miller_coop) d.pairs_per_item = 1;
  }
  d.job_lanes = k.job_lanes ? (uint32_t)k.job_lanes : 36u;
  // the scalars are allocated before the line decision below, so a line buffer
  // that ensure_or_release_lines gives up here is seen by that decision
  if (b->scalars && !b->on_device) {
    // staged with the other host arrays above
  } else if (b->scalars) {
    d.scalars = b->scalars;
  } else {
    // fresh 64-bit multipliers on the device: ChaCha20 keyed by 32 bytes of
    // getrandom() (+ 12-byte nonce) per call, rng.h
    uint32_t kn[11];
    random_bytes(kn, sizeof kn);
    if (int r = ensure_or_release_lines(c, c->scalars, n ? n : 1)) return r;
    launch_gen_scalars(c->st, kn, kn + 8, c->scalars.p, n);
    HIPCHK(hipGetLastError());
    d.scalars = c->scalars.p;
  }
  // fixed-argument lines (pairing.h miller_lines): the G2 half of the one-lane
  // Miller loop moves to the hash stream, phase 1 (C4 40.4 -> 39.5 ms); with
  // one pair per item it loses (C4/2 26.4 -> 28.5 ms)
  d.lines = (uint32_t)(!d.split && !d.miller_coop && (k.lines >= 0 ? k.lines : d.pairs_per_item >= 2));
  // the lines take 3 x 68 Fp2 = 19.6 KB per set (1.97 GB at C4, 2.6 GB at the
  // Node pool's 2^17-set batch cap): kept only while a quarter of the free HBM
  // covers them, else the loop recomputes them (miller_loop2, same values)
  if (d.lines) {
    const size_t need = (size_t)3 * MILLER_STEPS * n * sizeof(fp2_t);
    size_t free_b = 0, total_b = 0;
    if (need > c->lines.cap * sizeof(fp2_t) &&
        (hipMemGetInfo(&free_b, &total_b) != hipSuccess || need > free_b / 4))
      d.lines = 0;
  }
  // four pairs per item exist only over precomputed lines (miller_loop_lines4)
  if (d.pairs_per_item == 4 && !d.lines) d.pairs_per_item = 2;
  return 0;
}

static int work_alloc_once(bgv_ctx* c, const dev_batch& d, dev_work& w);

// a kept line buffer the batch does not use gives way under memory pressure
static int work_alloc(bgv_ctx* c, const dev_batch& d, dev_work& w) {
  int r = work_alloc_once(c, d, w);
  if (r && !d.lines && c->lines.cap) {
    c->lines.release();
    c->lines_idle = 0;
    r = work_alloc_once(c, d, w);
  }
  return r;
}

static int work_alloc_once(bgv_ctx* c, const dev_batch& d, dev_work& w) {
  const uint32_t n = d.n_sets, J = d.n_jobs;
  const size_t ns = n ? n : 1, nj = J ? J : 1;
  int r = 0;
  if ((r = c->chunk_off.ensure(ns + 1)) || (r = c->chunk_set.ensure((size_t)d.chunk_bound + 1)) ||
      (r = c->pk_part.ensure((size_t)d.chunk_bound + 1)))
    return r;
  w.chunk_off = c->chunk_off.p; w.chunk_set = c->chunk_set.p; w.pk_part = c->pk_part.p;
  if ((r = c->sig_aff.ensure(ns)) || (r = c->h_aff.ensure(ns)) || (r = c->sig_inf.ensure(ns)) ||
      (r = c->sig_code.ensure(ns)) || (r = c->pk_code.ensure(ns)) || (r = c->rpk_aff.ensure(ns)) ||
      (r = c->rsig.ensure(ns)) || (r = c->f_set.ensure(ns + nj)) || (r = c->set_code.ensure(ns)) ||
      (r = c->set_job.ensure(ns)) || (r = c->item_off.ensure(nj + 1)) || (r = c->item_job.ensure(ns + nj + 1)) || (r = c->f_job.ensure(nj)) || (r = c->f_batch.ensure(nj)) || (r = c->f_tmp.ensure(nj / 8 + 1)) ||
      (r = c->s_aff.ensure(nj)) || (r = c->s_inf.ensure(nj)) || (r = c->job_code.ensure(nj)) ||
      (r = c->job_result.ensure(nj)) || (r = c->f_part.ensure(4)) || (r = c->flags.ensure(8)))
    return r;
  w.sig_aff = c->sig_aff.p; w.h_aff = c->h_aff.p; w.sig_inf = c->sig_inf.p; w.sig_code = c->sig_code.p;
  w.pk_code = c->pk_code.p; w.rpk_aff = c->rpk_aff.p; w.rsig = c->rsig.p; w.f_set = c->f_set.p;
  w.set_code = c->set_code.p; w.f_job = c->f_job.p; w.job_code = c->job_code.p; w.job_result = c->job_result.p;
  w.f_part = c->f_part.p; w.flags = c->flags.p;
  w.item_off = c->item_off.p; w.item_job = c->item_job.p;
  w.set_job = c->set_job.p; w.f_batch = c->f_batch.p; w.f_tmp = c->f_tmp.p; w.s_aff = c->s_aff.p; w.s_inf = c->s_inf.p;
  w.q_part = nullptr; w.sig_grp = nullptr; w.pk_agg = nullptr;
  if (d.split) {
    if ((r = c->q_part.ensure(2 * ns)) || (r = c->sig_grp.ensure(ns))) return r;
    w.q_part = c->q_part.p; w.sig_grp = c->sig_grp.p;
  } else if (d.defer_grp) {
    if ((r = c->sig_grp.ensure(ns))) return r;
    w.sig_grp = c->sig_grp.p;
  }
  // the line buffer (19.6 KB per set, 1.3-2.6 GB) stays across batches: a
  // node alternating gossip batches with range-sync segments would otherwise
  // hipFree / hipMalloc gigabytes (each free synchronises the device) on every
  // switch; it goes back after LINES_KEEP batches in a row without lines
  static const uint32_t LINES_KEEP = 64;
  w.lines = nullptr;
  if (d.lines) {
    c->lines_idle = 0;
    if ((r = c->lines.ensure((size_t)3 * MILLER_STEPS * ns))) return r;
    w.lines = c->lines.p;
  } else if (c->lines.cap && ++c->lines_idle >= LINES_KEEP) {
    c->lines.release();
    c->lines_idle = 0;
  }
  w.msm_bucket = nullptr; w.msm_mask = nullptr; w.msm_win = nullptr;
  if (d.msm == 2) {
    if ((r = c->msm_bucket.ensure(nj * 16 * 15)) || (r = c->msm_mask.ensure(nj * 16)) || (r = c->msm_win.ensure(nj * 16))) return r;
    w.msm_bucket = c->msm_bucket.p; w.msm_mask = c->msm_mask.p; w.msm_win = c->msm_win.p;
  } else if (d.msm == 4) {
    if ((r = c->msm_win.ensure(nj * 16))) return r;
    w.msm_win = c->msm_win.p;
  }
  return 0;
}

// run stages [from, to) with an event before each
// Stage graph on three streams (the stages read disjoint inputs and write
// disjoint buffers, bgv_kernels.hip):
//   st      : sig -> sig_scale -> [pk] sig_sum_tree -> miller_loop_jobs -> [miller] tail
//   st_hash : hash -> [pk] miller_loop (the set pairs)
//   st_pk   : pk_gather -> pk_aggregate_scale   ([pk] = after pk_aggregate_scale)
// The set-pair Miller loops need only H(m) and the aggregated keys, so they
// start while the signatures are still being scaled: at C4 the Miller kernel
// fills 78% of the SIMDs (one wave each) and sig_scale takes the rest.
// Per-stage timing events (stats->stage_ms) cost ~5 us of queue time each on
// the critical path, so latency batches record only the stream dependencies
// (untimed events) and the total.
static int run_stages(bgv_ctx* c, const dev_batch& d, const dev_work& w, int from, int to) {
  const bool fork = from <= ST_SIG && to > ST_F_TREE;
  const bool timed = c->cfg.timing >= 0 ? c->cfg.timing != 0 : d.n_sets >= 65536;
  c->timed = timed;
  c->last_d = d;
  c->run_from = from;
  c->run_to = to;
  hipEvent_t* dep = timed ? c->ev_end : c->ev_dep;  // what the stream waits below wait on
  if (!timed && !(d.maps_early && from == 0)) HIPCHK(hipEventRecord(c->ev[from], c->st));
  // latency batches fork the hash leg BEFORE the index set-up: hash_to_G2 reads
  // only the messages and heads the critical path (hash -> Miller -> fold ->
  // final exp); large batches keep the set-up alone on the GPU (its
  // one-workgroup scan starves under the bulk kernels).  At C4 the signature
  // decode is dispatched first, on the set-up's own stream: dispatching the
  // hash first ends it at ~12.5 instead of ~16.3 ms, but the signature chain
  // (decode -> MSM buckets -> window sums -> job pairs, ~32 ms of the 37)
  // then runs into the Miller phase, and the step lost 0.2-3.8 ms in every
  // order tried (profiles/r05m_bulk_stage_order.txt)
  const bool early_hash = fork && d.split && from <= ST_HASH && to > ST_HASH;
  auto launch_one = [&](int s) -> int {
    hipStream_t st = c->st;
    // fixed-argument lines: right behind the hash on its stream, before the
    // Miller stage waits for the pubkeys (timed in neither stage)
    if (s == ST_MILLER && d.lines) {
      launch_lines(fork ? c->st_hash : c->st, d, w);  // bgv_miller.hip
      HIPCHK(hipGetLastError());
    }
    if (fork) {
      if (s == ST_HASH || s == ST_MILLER) st = c->st_hash;
      if (s == ST_PK || s == ST_PK_SCALE) st = c->st_pk;
      if (s == ST_S_TREE || s == ST_MILLER) HIPCHK(hipStreamWaitEvent(st, dep[ST_PK_SCALE], 0));
      if (s == ST_F_TREE) HIPCHK(hipStreamWaitEvent(st, dep[ST_MILLER], 0));
    }
    // maps launched early on st_hash: a hash stage on another stream (a run
    // that does not fork, e.g. bgv_debug_stages' first range) waits for them
    if (s == ST_HASH && d.maps_early && st != c->st_hash) HIPCHK(hipStreamWaitEvent(st, c->ev_maps, 0));
    if (timed) HIPCHK(hipEventRecord(c->ev[s], st));
    // deferred subgroup checks: their verdicts enter the codes before the fold
    if (s == ST_F_TREE && d.defer_grp) {
      if (fork) HIPCHK(hipStreamWaitEvent(st, c->ev_grp, 0));
      launch_sig_fixup(st, d, w);
    }
    launch_stage(st, s, d, w);
    HIPCHK(hipGetLastError());
    if (timed) HIPCHK(hipEventRecord(c->ev_end[s], st));
    else if (fork && (s == ST_PK_SCALE || s == ST_HASH || s == ST_MILLER)) HIPCHK(hipEventRecord(c->ev_dep[s], st));
    if (d.defer_grp && s == ST_SIG && fork) HIPCHK(hipEventRecord(c->ev_sigdec, st));
    if (d.defer_grp && s == ST_PK_SCALE) {
      // the checks start once the Miller loops have their keys, beside them;
      // BGV_CHK_STREAM: on a low-priority stream of their own, so the waves of
      // the hash stream (the fixed-argument lines, then the Miller loops) are
      // dispatched first when slots free up
      // (latency-mode batches only: at C4 the checks on the pubkey stream measured
      // 0.3 ms faster, 4 same-box rounds, profiles/r04z_ab_chk_c4.txt)
      hipStream_t cs = st;
      if (fork && BGV_CHK_STREAM && d.split) {
        HIPCHK(hipEventRecord(c->ev_chk, st));
        cs = c->st_chk;
        HIPCHK(hipStreamWaitEvent(cs, c->ev_chk, 0));
      }
      if (fork) HIPCHK(hipStreamWaitEvent(cs, c->ev_sigdec, 0));
      launch_sig_check(cs, d, w);
      HIPCHK(hipGetLastError());
      if (fork) HIPCHK(hipEventRecord(c->ev_grp, cs));
    }
    return 0;
  };
  if (early_hash) {  // enqueued first, so the host's launch latency does not delay it either
    HIPCHK(hipEventRecord(c->ev_fork, c->st));
    HIPCHK(hipStreamWaitEvent(c->st_hash, c->ev_fork, 0));
    if (int r = launch_one(ST_HASH)) return r;
  }
  if (from <= ST_PK) {
    launch_prep(c->st, d, w);
    HIPCHK(hipGetLastError());
  }
  if (fork) {
    HIPCHK(hipEventRecord(c->ev_prep, c->st));
    if (!early_hash) HIPCHK(hipStreamWaitEvent(c->st_hash, c->ev_prep, 0));
    HIPCHK(hipStreamWaitEvent(c->st_pk, c->ev_prep, 0));
  }
  for (int s = from; s < to; s++)
    if (!(early_hash && s == ST_HASH))
      if (int r = launch_one(s)) return r;
  HIPCHK(hipEventRecord(c->ev[to], c->st));
  return 0;
}

static void stats_layout(bgv_stats* s, const dev_batch& d) {
  s->split = d.split;
  s->miller_lanes = d.miller_coop ? d.miller_coop : 1u;
  s->pairs_per_item = d.pairs_per_item;
  s->msm = d.msm;
  s->lines = d.lines;
  s->defer_from = d.defer_grp ? d.defer_from : d.n_sets;
  s->clear_lanes = d.clear_lanes;
  s->miller_kv = d.miller_kv;
}

// job results, set codes and the batch flag through pinned memory; the
// lodestar_bls_thread_pool_* counters from the host view of the offsets
static int finish_results(bgv_ctx* c, const dev_batch& d, const dev_work& w, int32_t* job_result, int32_t* set_code,
                          bgv_stats* stats) {
  const size_t jr_off = 256, sc_off = jr_off + (((size_t)d.n_jobs * 4 + 255) & ~size_t(255));
  const bool want_sc = set_code && d.n_sets;
  if (int r = pinned_reserve(c->pin_out, c->pin_out_cap, sc_off + (want_sc ? (size_t)d.n_sets * 4 : 0))) return r;
  if (d.n_jobs) HIPCHK(hipMemcpyAsync(c->pin_out + jr_off, w.job_result, (size_t)d.n_jobs * 4, hipMemcpyDeviceToHost, c->st));
  if (want_sc) HIPCHK(hipMemcpyAsync(c->pin_out + sc_off, w.set_code, (size_t)d.n_sets * 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipMemcpyAsync(c->pin_out, w.flags, 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  c->staged_pending = false;
  uint32_t flag = 0;
  memcpy(&flag, c->pin_out, 4);
  if (d.n_jobs) memcpy(job_result, c->pin_out + jr_off, (size_t)d.n_jobs * 4);
  if (want_sc) memcpy(set_code, c->pin_out + sc_off, (size_t)d.n_sets * 4);
  if (stats) {
    memset(stats, 0, sizeof *stats);
    if (c->timed)
      for (int s = 0; s < ST_COUNT && s < BGV_N_STAGES; s++) HIPCHK(hipEventElapsedTime(&stats->stage_ms[s], c->ev[s], c->ev_end[s]));
    HIPCHK(hipEventElapsedTime(&stats->total_ms, c->ev[0], c->ev[ST_COUNT]));
    stats->n_sets = d.n_sets;
    stats->n_jobs = d.n_jobs;
    stats_layout(stats, d);
    uint32_t valid_jobs = 0, valid_sets = 0;
    const uint32_t* jo = c->jo_host.data();
    for (uint32_t j = 0; j < d.n_jobs; j++)
      if (job_result[j] >= 0) { valid_jobs++; valid_sets += jo[j + 1] - jo[j]; }
    stats->pubkeys_aggregated = c->pk_total;
    stats->batch_retries = (valid_jobs && !flag) ? 1u : 0u;
    stats->batch_sigs_success = flag ? valid_sets : 0u;
  }
  return 0;
}

int bgv_last_stats(bgv_ctx* c, bgv_stats* stats) {
  if (!c || !stats) return fail(BGV_E_INVALID_ARG, "null argument");
  memset(stats, 0, sizeof *stats);
  if (c->run_to <= c->run_from) return BGV_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipEventSynchronize(c->ev[c->run_to]));
  if (c->timed)
    for (int s = c->run_from; s < c->run_to && s < BGV_N_STAGES; s++) HIPCHK(hipEventElapsedTime(&stats->stage_ms[s], c->ev[s], c->ev_end[s]));
  HIPCHK(hipEventElapsedTime(&stats->total_ms, c->ev[c->run_from], c->ev[c->run_to]));
  stats_layout(stats, c->last_d);
  return BGV_OK;
}

int bgv_verify(bgv_ctx* c, const bgv_batch* b, int32_t* job_result, int32_t* set_code, bgv_stats* stats) {
  if (!c || !b || (!job_result && b->n_jobs)) return fail(BGV_E_INVALID_ARG, "null argument");
  c->partial_pending = false;
  HIPCHK(hipSetDevice(c->device));
  active_guard ag(c->device);
  dev_batch d;
  if (int r = prepare(c, b, d, true)) return r;
  dev_work w;
  if (int r = work_alloc(c, d, w)) return r;
  if (int r = run_stages(c, d, w, 0, ST_COUNT)) return r;
  return finish_results(c, d, w, job_result, set_code, stats);
}

// ---- multi-GPU partials ---------------------------------------------------
// fp12 (plain limbs, already out of Montgomery form on the device) <-> 576 B
static void fp12_plain_to_bytes(uint8_t* out, const fp12_t& f) {
  const fp2_t* cs[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  for (int k = 0; k < 6; k++) {
    fp_to_be48(out + 96 * k, cs[k]->c0);
    fp_to_be48(out + 96 * k + 48, cs[k]->c1);
  }
}

static void fp12_plain_from_bytes(fp12_t& f, const uint8_t* in) {
  fp2_t* cs[6] = {&f.c0.c0, &f.c1.c0, &f.c0.c1, &f.c1.c1, &f.c0.c2, &f.c1.c2};
  for (int k = 0; k < 6; k++) {
    fp_from_be48(cs[k]->c0, in + 96 * k);
    fp_from_be48(cs[k]->c1, in + 96 * k + 48);
  }
}

int bgv_partial(bgv_ctx* c, const bgv_batch* b, uint8_t* miller576, int32_t* set_code, int32_t* job_result,
                int32_t* ok_out) {
  if (!c || !b || !miller576) return fail(BGV_E_INVALID_ARG, "null argument");
  c->partial_pending = false;
  HIPCHK(hipSetDevice(c->device));
  active_guard ag(c->device);
  dev_batch d;
  if (int r = prepare(c, b, d, true)) return r;
  dev_work w;
  if (int r = work_alloc(c, d, w)) return r;
  if (int r = run_stages(c, d, w, ST_SIG, ST_BATCH_FINAL)) return r;
  launch_stage(c->st, ST_SET_CODES, d, w);
  fp12_t f;
  if (d.n_jobs) {
    launch_fp12_convert(c->st, w.f_batch, w.f_part, 1, false);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&f, w.f_part, sizeof f, hipMemcpyDeviceToHost, c->st));
  } else {
    memset(&f, 0, sizeof f);
    f.c0.c0.c0.l[0] = 1;  // plain 1
  }
  std::vector<int32_t> jc(d.n_jobs ? d.n_jobs : 1);
  if (d.n_jobs) HIPCHK(hipMemcpyAsync(jc.data(), w.job_code, (size_t)d.n_jobs * 4, hipMemcpyDeviceToHost, c->st));
  if (set_code && d.n_sets) HIPCHK(hipMemcpyAsync(set_code, w.set_code, (size_t)d.n_sets * 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  c->staged_pending = false;
  fp12_plain_to_bytes(miller576, f);
  int32_t ok = 1;
  for (uint32_t j = 0; j < d.n_jobs; j++) {
    if (jc[j] != 0) ok = 0;
    if (job_result) job_result[j] = jc[j] != 0 ? -jc[j] : 1;
  }
  if (ok_out) *ok_out = ok;
  c->part_d = d;
  c->part_w = w;
  c->partial_pending = true;
  return BGV_OK;
}

int bgv_partial_finish(bgv_ctx* c, int32_t* job_result, bgv_stats* stats) {
  if (!c) return fail(BGV_E_INVALID_ARG, "null ctx");
  if (!c->partial_pending) return fail(BGV_E_STATE, "bgv_partial_finish needs bgv_partial as the previous call on the context");
  const dev_batch& d = c->part_d;
  const dev_work& w = c->part_w;
  if (!job_result && d.n_jobs) return fail(BGV_E_INVALID_ARG, "null argument");
  c->partial_pending = false;
  HIPCHK(hipSetDevice(c->device));
  c->timed = false;
  c->run_from = 0;
  c->run_to = ST_COUNT;
  HIPCHK(hipEventRecord(c->ev[0], c->st));
  launch_stage(c->st, ST_BATCH_FINAL, d, w);
  launch_stage(c->st, ST_JOB_FINAL, d, w);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[ST_COUNT], c->st));
  return finish_results(c, d, w, job_result, nullptr, stats);
}

// (keeps a pending bgv_partial state: the dist flow is partial -> combine ->
// partial_finish; the combination touches only f_part and its own flag word)
int bgv_combine_final(bgv_ctx* c, const uint8_t* parts, uint32_t n, int32_t* is_one) {
  if (!c || (!parts && n) || !is_one) return fail(BGV_E_INVALID_ARG, "null argument");
  HIPCHK(hipSetDevice(c->device));
  std::vector<fp12_t> h(n ? n : 1);
  for (uint32_t k = 0; k < n; k++) fp12_plain_from_bytes(h[k], parts + 576u * k);
  if (int r = c->f_part.ensure(2 * (size_t)n + 65)) return r;
  if (int r = c->flags.ensure(8)) return r;
  if (n) HIPCHK(hipMemcpyAsync(c->f_part.p + n, h.data(), (size_t)n * sizeof(fp12_t), hipMemcpyHostToDevice, c->st));
  launch_fp12_convert(c->st, c->f_part.p + n, c->f_part.p, n, true);
  launch_combine_final(c->st, c->f_part.p, n, c->flags.p + 4);
  HIPCHK(hipGetLastError());
  uint32_t flag = 0;
  HIPCHK(hipMemcpyAsync(&flag, c->flags.p + 4, 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  *is_one = flag ? 1 : 0;
  return BGV_OK;
}

// ---- test-only: per-stage intermediates -------------------------------------
int bgv_debug_stages(bgv_ctx* c, const bgv_batch* b, int32_t* job_result, int32_t* set_code, bgv_debug* o) {
  if (!c || !b || !o || (!job_result && b->n_jobs)) return fail(BGV_E_INVALID_ARG, "null argument");
  c->partial_pending = false;
  HIPCHK(hipSetDevice(c->device));
  dev_batch d;
  if (int r = prepare(c, b, d, true)) return r;
  dev_work w;
  if (int r = work_alloc(c, d, w)) return r;
  const uint32_t n = d.n_sets, J = d.n_jobs;
  if (int r = c->pk_agg.ensure(n ? n : 1)) return r;
  w.pk_agg = c->pk_agg.p;
  // the Miller values are copied before the product tree, which folds groups
  // of them in place (k_job_prefold, k_f_level); deferred subgroup verdicts
  // are applied first (idempotent: the tree stage applies them again)
  if (int r = run_stages(c, d, w, 0, ST_F_TREE)) return r;
  if (d.defer_grp) launch_sig_fixup(c->st, d, w);
  if (int r = c->dbg_f.ensure((size_t)n + J + 1)) return r;
  if (n + J) HIPCHK(hipMemcpyAsync(c->dbg_f.p, w.f_set, (size_t)(n + J) * sizeof(fp12_t), hipMemcpyDeviceToDevice, c->st));
  if (int r = run_stages(c, d, w, ST_F_TREE, ST_COUNT)) return r;
  // final exponentiations of every Miller value, job product and the batch product
  const uint32_t n_fe = n + 2 * J + 1;
  if (int r = c->dbg_fe.ensure(n_fe)) return r;
  launch_final_exp_many(c->st, c->dbg_f.p, c->dbg_fe.p, n + J);
  launch_final_exp_many(c->st, w.f_job, c->dbg_fe.p + n + J, J);
  if (J) launch_final_exp_many(c->st, w.f_batch, c->dbg_fe.p + n + 2 * J, 1);
  launch_fp12_convert(c->st, c->dbg_fe.p, c->dbg_fe.p, n_fe, false);
  HIPCHK(hipGetLastError());
  struct part { uint8_t* host; size_t bytes; } parts[8];
  int np = 0;
  size_t off = 0;
  auto add = [&](uint8_t* host, size_t bytes) -> uint8_t* {
    const size_t o2 = off;
    off += (bytes + 255) & ~size_t(255);
    parts[np++] = {host, bytes};
    return (uint8_t*)o2;  // offset, rebased below
  };
  uint8_t* o_sig = add(o->sig_aff, (size_t)n * 192);
  uint8_t* o_h = add(o->h_aff, (size_t)n * 192);
  uint8_t* o_pk = add(o->pk_agg, (size_t)n * 96);
  uint8_t* o_rpk = add(o->rpk_aff, (size_t)n * 96);
  uint8_t* o_s = add(o->s_aff, (size_t)J * 192);
  if (int r = c->dbg_out.ensure(off ? off : 1)) return r;
  uint8_t* base = c->dbg_out.p;
  launch_export_g2a(c->st, w.sig_aff, base + (size_t)o_sig, n);
  launch_export_g2a(c->st, w.h_aff, base + (size_t)o_h, n);
  launch_export_g1a(c->st, w.pk_agg, base + (size_t)o_pk, n);
  launch_export_g1a(c->st, w.rpk_aff, base + (size_t)o_rpk, n);
  launch_export_g2a(c->st, w.s_aff, base + (size_t)o_s, J);
  HIPCHK(hipGetLastError());
  size_t pos = 0;
  for (int k = 0; k < np; k++) {
    if (parts[k].host && parts[k].bytes) HIPCHK(hipMemcpyAsync(parts[k].host, base + pos, parts[k].bytes, hipMemcpyDeviceToHost, c->st));
    pos += (parts[k].bytes + 255) & ~size_t(255);
  }
  std::vector<fp12_t> fe(n_fe);
  HIPCHK(hipMemcpyAsync(fe.data(), c->dbg_fe.p, (size_t)n_fe * sizeof(fp12_t), hipMemcpyDeviceToHost, c->st));
  if (int r = finish_results(c, d, w, job_result, set_code, nullptr)) return r;
  if (o->pair_fe)
    for (uint32_t k = 0; k < n + J; k++) fp12_plain_to_bytes(o->pair_fe + 576u * k, fe[k]);
  if (o->job_fe)
    for (uint32_t k = 0; k < J; k++) fp12_plain_to_bytes(o->job_fe + 576u * k, fe[n + J + k]);
  if (o->batch_fe) {
    if (J) fp12_plain_to_bytes(o->batch_fe, fe[n + 2 * J]);
    else memset(o->batch_fe, 0, 576);
  }
  return BGV_OK;
}

// ---- synthetic data --------------------------------------------------------
int bgv_gen_keys(bgv_ctx* c, uint32_t first, uint32_t n, uint64_t seed) {
  if (!c) return fail(BGV_E_INVALID_ARG, "null ctx");
  c->partial_pending = false;
  if (n == 0) return BGV_OK;
  if ((uint64_t)first + n > TABLE_MAX) return fail(BGV_E_TABLE_RANGE, "rows [%u, %llu) exceed the table limit 2^31 - 1", first, (unsigned long long)first + n);
  if (first > c->table_n) return fail(BGV_E_TABLE_RANGE, "row %u would leave a gap after the %u rows of the table", first, c->table_n);
  HIPCHK(hipSetDevice(c->device));
  if (int r = table_reserve(c, first + n)) return r;
  if (c->sk.cap < (size_t)(first + n) * 8) {
    // keep previously generated keys when growing
    dbuf<uint32_t> nb;
    if (int r = nb.ensure((size_t)(first + n) * 8)) return r;
    HIPCHK(hipMemsetAsync(nb.p, 0, nb.cap * 4, c->st));
    if (c->sk.p) HIPCHK(hipMemcpyAsync(nb.p, c->sk.p, c->sk.cap * 4, hipMemcpyDeviceToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    c->sk.release();
    c->sk = nb;
  }
  launch_gen_keys(c->st, c->table, c->sk.p, first, n, seed);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->st));
  if (first + n > c->table_n) c->table_n = first + n;
  return BGV_OK;
}

int bgv_gen_sign(bgv_ctx* c, const bgv_batch* b, uint8_t* sigs_out) {
  if (!c || !b || !sigs_out) return fail(BGV_E_INVALID_ARG, "null argument");
  if (!c->sk.p) return fail(BGV_E_INVALID_ARG, "bgv_gen_keys has not run on this context");
  HIPCHK(hipSetDevice(c->device));
  c->partial_pending = false;
  dev_batch d;
  bgv_batch bb = *b;
  bb.scalars = nullptr;
  if (int r = prepare(c, &bb, d, false)) return r;
  uint8_t* out = sigs_out;
  if (!b->on_device) {
    if (int r = c->gen_out.ensure((size_t)d.n_sets * 192 + 1)) return r;
    HIPCHK(hipMemsetAsync(c->gen_out.p, 0, (size_t)d.n_sets * 192, c->st));
    out = c->gen_out.p;
  }
  launch_gen_sign(c->st, d, c->sk.p, out);
  HIPCHK(hipGetLastError());
  if (!b->on_device) HIPCHK(hipMemcpyAsync(sigs_out, out, (size_t)d.n_sets * 192, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return BGV_OK;
}

// ---- field self-test ---------------------------------------------------------
int bgv_debug_fp_ops(bgv_ctx* c, const uint32_t* ab_in, uint32_t n, uint32_t* out) {
  if (!c || (n && (!ab_in || !out))) return fail(BGV_E_INVALID_ARG, "null argument");
  if (n > (1u << 20)) return fail(BGV_E_INVALID_ARG, "at most 2^20 operand pairs");
  if (!n) return BGV_OK;
  HIPCHK(hipSetDevice(c->device));
  if (int r = c->mb_fp.ensure((size_t)n * (2 + BGV_FP_OPS_N))) return r;
  fp_t* d_ab = c->mb_fp.p;
  fp_t* d_out = d_ab + (size_t)n * 2;
  HIPCHK(hipMemcpyAsync(d_ab, ab_in, (size_t)n * 2 * sizeof(fp_t), hipMemcpyHostToDevice, c->st));
  launch_fp_ops(c->st, d_ab, d_out, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, d_out, (size_t)n * BGV_FP_OPS_N * sizeof(fp_t), hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return BGV_OK;
}

int bgv_debug_g2_decode(bgv_ctx* c, const uint8_t* sigs192, const uint32_t* sig_len, uint32_t n, uint8_t* out192,
                        int32_t* codes) {
  if (!c || (n && (!sigs192 || !sig_len || !out192 || !codes))) return fail(BGV_E_INVALID_ARG, "null argument");
  if (n > (1u << 20)) return fail(BGV_E_INVALID_ARG, "at most 2^20 encodings");
  if (!n) return BGV_OK;
  HIPCHK(hipSetDevice(c->device));
  const size_t bytes = (size_t)n * (192 + 4 + 192 + 4);
  if (int r = c->dbg_out.ensure(bytes)) return r;
  uint8_t* d_sig = c->dbg_out.p;
  uint32_t* d_len = (uint32_t*)(d_sig + (size_t)n * 192);
  uint8_t* d_out = (uint8_t*)(d_len + n);
  int32_t* d_code = (int32_t*)(d_out + (size_t)n * 192);
  HIPCHK(hipMemcpyAsync(d_sig, sigs192, (size_t)n * 192, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipMemcpyAsync(d_len, sig_len, (size_t)n * 4, hipMemcpyHostToDevice, c->st));
  launch_g2_decode_dbg(c->st, d_sig, d_len, d_out, d_code, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out192, d_out, (size_t)n * 192, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipMemcpyAsync(codes, d_code, (size_t)n * 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return BGV_OK;
}

// ---- microbenchmarks ---------------------------------------------------------
int bgv_bench_fpmul(bgv_ctx* c, uint32_t lanes, uint32_t iters, float* ms) {
  if (!c || !ms || lanes == 0 || lanes % 256) return fail(BGV_E_INVALID_ARG, "lanes must be a positive multiple of 256");
  HIPCHK(hipSetDevice(c->device));
  if (int r = c->mb_fp.ensure((size_t)lanes * 2)) return r;
  std::vector<fp_t> h((size_t)lanes * 2);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (auto& e : h) {
    for (int k = 0; k < NL; k++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; e.l[k] = (uint32_t)x; }
    e.l[NL - 1] &= 0x0fffffffu;  // < p
  }
  HIPCHK(hipMemcpyAsync(c->mb_fp.p, h.data(), h.size() * sizeof(fp_t), hipMemcpyHostToDevice, c->st));
  launch_bench_fpmul(c->st, c->mb_fp.p, lanes, 16);  // warm-up
  HIPCHK(hipEventRecord(c->ev[0], c->st));
  launch_bench_fpmul(c->st, c->mb_fp.p, lanes, iters);
  HIPCHK(hipEventRecord(c->ev[1], c->st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventSynchronize(c->ev[1]));
  HIPCHK(hipEventElapsedTime(ms, c->ev[0], c->ev[1]));
  return BGV_OK;
}

int bgv_bench_mad(bgv_ctx* c, uint32_t lanes, uint32_t iters, float* ms) {
  if (!c || !ms || lanes == 0 || lanes % 256) return fail(BGV_E_INVALID_ARG, "lanes must be a positive multiple of 256");
  HIPCHK(hipSetDevice(c->device));
  if (int r = c->mb_u64.ensure(lanes)) return r;
  HIPCHK(hipMemsetAsync(c->mb_u64.p, 0x5a, (size_t)lanes * 8, c->st));
  launch_bench_mad(c->st, c->mb_u64.p, lanes, 16);
  HIPCHK(hipEventRecord(c->ev[0], c->st));
  launch_bench_mad(c->st, c->mb_u64.p, lanes, iters);
  HIPCHK(hipEventRecord(c->ev[1], c->st));
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventSynchronize(c->ev[1]));
  HIPCHK(hipEventElapsedTime(ms, c->ev[0], c->ev[1]));
  return BGV_OK;
}

