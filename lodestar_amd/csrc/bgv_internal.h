// Internal interface between the kernels (bgv_kernels.hip) and the host
// orchestration behind the C ABI (bgv_api.hip).  Not installed.
#pragma once
#include "pairing.h"
#include "rng.h"

namespace bgv {

// internal per-set codes beyond blst's (see include/bgv.h bgv_set_code)
enum : int32_t {
  C_INDEX_RANGE = 9,
  C_EMPTY_JOB = 10,
};

// HBM layout of one batch (device pointers).  All arrays are dense and
// indexed by set (or job); see include/bgv.h bgv_batch for their meaning.
struct dev_batch {
  uint32_t n_sets, n_jobs, n_raw, table_n;
  uint32_t span_log2;    // per-job reduction tree covers 2^span_log2 sets
  uint32_t chunk_bound;  // upper bound of pubkey chunks (grid of k_pk_chunk)
  uint32_t miller_coop;     // set pairs: 0 one-lane Miller loop (k_miller), 2 / 4 the two- / four-lane loop
                            // (k_miller_duo / k_miller_quad), else lanes per pair of the cooperative loop (miller_coop.h: 6, 18 or 36)
  uint32_t job_lanes;       // (-G1, S_job) pairs: lanes per pair of the cooperative loop (6, 18 or 36)
  uint32_t pairs_per_item;  // Miller pairs sharing one accumulator (1, or 2 for batches that fill the GPU)
  uint32_t msm;             // sum r_i sigma_i: 0 per-set [r_i] sigma_i + tree (latency mode: cooperative, with the checks),
                            // 1 per-job fused MSM (k_msm_fused), 2 (job, window)-lane MSM (k_msm_bucket), 3 one-lane per-set
                            // scaling + tree with the subgroup checks deferred (latency-mode hash), 4 (job, window,
                            // digit)-lane MSM (k_msm_digit)
  uint32_t split;           // 1: latency mode: hash maps on two lanes per set, subgroup check beside [r_i] sigma_i
  uint32_t clear_lanes;     // latency mode: lanes per point of the cofactor clearing (9, or 3)
  uint32_t miller_kv;       // latency mode: 0, or the slots S of the two-pair Miller loop in views (k_miller_kv, 3 S lanes)
  uint32_t maps_early;      // latency mode: k_hash_map already launched by prepare() (bgv_api.hip early_maps)
  uint32_t prefold_log2;    // >0: two-level job fold, groups of 2^prefold_log2 sets (k_job_prefold); 0: one level
  uint32_t lines;           // one-lane Miller loop over fixed-argument lines: the hash stream stores every set's
                            // 68 unevaluated lines (launch_lines), k_miller evaluates them at P (pairing.h)
  uint32_t defer_from;      // defer_grp: sets below it are checked in ST_SIG as usual, the rest later (multiple of 64)
  uint32_t defer_grp;       // bulk mode: ST_SIG only decodes; the G2 subgroup check runs beside the Miller loops
                            // (launch_sig_check) and its verdicts reach the job codes before the fold (launch_sig_fixup)
  const uint32_t* job_off;
  const uint32_t* pk_off;
  const uint32_t* pk_idx;
  const g1a* raw_pks;  // Montgomery affine (converted by k_raw_pks)
  const g1a* table;    // index2pubkey, Montgomery affine, 96 B per validator
  const uint8_t* msgs;
  const uint8_t* sigs;
  const uint32_t* sig_len;
  const uint64_t* scalars;
};

// Per-batch intermediates resident in HBM.
struct dev_work {
  g2a* sig_aff;       // decoded signature (affine)
  uint32_t* sig_inf;  // signature is the identity
  int32_t* sig_code;  // parse / subgroup outcome
  g2a* h_aff;         // H(m)
  g2j* q_part;        // [2 n_sets] split mode: the two mapped points of every message
  uint32_t* sig_grp;  // split / defer_grp mode: signature passed the subgroup check
  g2j* msm_bucket;    // [n_jobs * 16 windows * 15 buckets] (msm = 2)
  uint32_t* msm_mask; // [n_jobs * 16] occupied buckets of each (job, window)
  g2j* msm_win;       // [n_jobs * 16] window sums (msm = 2, 4)
  uint32_t* chunk_off;  // [n_sets + 1] scan of per-set pubkey chunk counts
  uint32_t* chunk_set;  // set of every chunk
  g1j* pk_part;         // per-chunk partial sums
  g1a* rpk_aff;       // [r_i] aggregated pubkey, affine
  g1a* pk_agg;        // aggregated pubkey before scaling, affine (bgv_debug_stages only; else NULL)
  int32_t* pk_code;
  g2j* rsig;          // [r_i] sigma_i
  uint32_t* set_job;  // job id of every set
  uint32_t* item_off; // [n_jobs + 1] scan of Miller work items per job (2 sets each)
  uint32_t* item_job; // job of every Miller work item
  g2a* s_aff;         // per job: sum [r_i] sigma_i, affine
  uint32_t* s_inf;
  fp2_t* lines;       // [68 steps][3][n_sets] unevaluated Miller lines of H(m_i) (dev_batch.lines)
  fp12_t* f_set;      // per pair Miller value: n_sets set pairs, then n_jobs (-G1, S_job) pairs
  fp12_t* f_job;      // per-job Miller product (incl. the -G1 pair)
  fp12_t* f_batch;    // batch product scratch [n_jobs]; the product ends in f_batch[0]
  fp12_t* f_tmp;      // batch fold ping-pong [ceil(n_jobs / 8)]
  int32_t* job_code;
  int32_t* job_result;
  int32_t* set_code;
  fp12_t* f_part;     // conversion scratch for partials
  uint32_t* flags;    // [0] = whole batch verified
};

enum Stage {
  ST_SIG = 0,
  ST_HASH,
  ST_PK,        // chunked gather + partial sums from the HBM table (k_pk_chunk)
  ST_PK_SCALE,  // per set: fold the chunk sums, [r_i] PK_i, affine (k_pk)
  ST_SIG_SCALE,
  ST_S_TREE,
  ST_MILLER,
  ST_MILLER_JOBS,
  ST_F_TREE,
  ST_BATCH_PROD,
  ST_BATCH_FINAL,
  ST_JOB_FINAL,
  ST_SET_CODES,
  ST_COUNT
};

#ifdef __HIPCC__
BGV_HD bool g1a_is_zero(const g1a& p) { return fp_is_zero(p.x) && fp_is_zero(p.y); }

// row of the pubkey table (or of the raw side table for bit 31); an index
// past either flags range_err and yields the identity
__device__ __forceinline__ void load_pk(g1a& out, const dev_batch& b, uint32_t idx, bool& range_err) {
  if (idx & 0x80000000u) {
    const uint32_t r = idx & 0x7fffffffu;
    if (r >= b.n_raw) { range_err = true; fp_set_zero(out.x); fp_set_zero(out.y); return; }
    out = b.raw_pks[r];
  } else {
    if (idx >= b.table_n) { range_err = true; fp_set_zero(out.x); fp_set_zero(out.y); return; }
    out = b.table[idx];
  }
}
#endif

// keys per chunk of the balanced pubkey gather (k_pk_chunk)
constexpr uint32_t PK_CHUNK = 32;

void launch_pk_gather(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_gather.hip
void launch_raw_pks(hipStream_t st, const uint8_t* raw, g1a* out, uint32_t n);
void launch_table_from_compressed(hipStream_t st, const uint8_t* in, g1a* out, uint32_t n, int32_t* codes);
void launch_table_from_uncompressed(hipStream_t st, const uint8_t* in, g1a* out, uint32_t n, int32_t* codes);
void launch_table_export(hipStream_t st, const g1a* tab, uint8_t* out, uint32_t n);
void launch_pk_validate(hipStream_t st, const uint8_t* in, uint32_t n, int32_t* codes);
void launch_hash_maps(hipStream_t st, const dev_batch& b, const dev_work& w);  // prepare(): before the set-up
void launch_prep(hipStream_t st, const dev_batch& b, const dev_work& w);  // before ST_PK / ST_MILLER
void launch_stage(hipStream_t st, int stage, const dev_batch& b, const dev_work& w);
void launch_miller(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_miller.hip
void launch_lines(hipStream_t st, const dev_batch& b, const dev_work& w);   // bgv_miller.hip
void launch_miller_duo(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_miller.hip
void launch_miller_quad(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_miller.hip
void launch_sig_check(hipStream_t st, const dev_batch& b, const dev_work& w);   // subgroup checks only (sig_grp)
void launch_sig_fixup(hipStream_t st, const dev_batch& b, const dev_work& w);   // k_sig_fix + k_job_recode
void launch_sig_split_coop(hipStream_t st, const dev_batch& b, const dev_work& w);   // bgv_latency.hip
void launch_hash_clear_coop(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_latency.hip
void launch_hash_clear_trio(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_latency.hip
void launch_s_level_coop(hipStream_t st, const dev_batch& b, const dev_work& w, uint32_t s);  // bgv_latency.hip
void launch_msm_job_coop(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_latency.hip
void launch_pk_coop(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_latency.hip
void launch_miller_kv(hipStream_t st, const dev_batch& b, const dev_work& w);  // bgv_miller.hip
void launch_fp12_tail(hipStream_t st, int stage, const dev_batch& b, const dev_work& w);  // bgv_tail.hip
void launch_combine_final(hipStream_t st, const fp12_t* parts, uint32_t n, uint32_t* flag);
void launch_final_exp_many(hipStream_t st, const fp12_t* in, fp12_t* out, uint32_t n);  // bgv_debug_stages
void launch_export_g1a(hipStream_t st, const g1a* in, uint8_t* out96, uint32_t n);
void launch_export_g2a(hipStream_t st, const g2a* in, uint8_t* out192, uint32_t n);
void launch_fp12_convert(hipStream_t st, const fp12_t* in, fp12_t* out, uint32_t n, bool to_mont);
void launch_gen_keys(hipStream_t st, g1a* table, uint32_t* sk, uint32_t first, uint32_t n, uint64_t seed);
void launch_gen_sign(hipStream_t st, const dev_batch& b, const uint32_t* sk, uint8_t* out);
void launch_fp_ops(hipStream_t st, const fp_t* ab, fp_t* out, uint32_t n);
void launch_g2_decode_dbg(hipStream_t st, const uint8_t* sigs192, const uint32_t* sig_len, uint8_t* out192, int32_t* codes,
                         uint32_t n);
void launch_bench_fpmul(hipStream_t st, fp_t* io, uint32_t lanes, uint32_t iters);
void launch_gen_scalars(hipStream_t st, const uint32_t key[8], const uint32_t nonce[3], uint64_t* out, uint32_t n);
void launch_bench_mad(hipStream_t st, uint64_t* io, uint32_t lanes, uint32_t iters);

}  // namespace bgv
