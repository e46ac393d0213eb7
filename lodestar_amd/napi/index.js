"use strict";
// IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-51) over
// the N-API addon, in plain CommonJS so it runs on the Node in this image.
// The TypeScript class a maintainer adds (INTEGRATION.md section 4) has the
// same shape; this file is what the addon's tests drive.
//
// It keeps the pool contract of BlsMultiThreadWorkerPool
// (multithread/index.ts:120-431) with the GPU context in the role of the
// worker:
//  * every call is chunked into jobs of <= 128 sets (chunkifyMaximizeChunkSize);
//  * batchable jobs wait in a buffer flushed after 100 ms or as soon as more
//    than 32 signature sets are buffered (queueBlsWork, index.ts:262-291);
//  * non-batchable jobs are queued and started on the next macro task;
//  * an idle context takes every queued job (a GPU wants one large batch; the
//    CPU pool packs <= 128 sets per worker message), and the library's
//    whole-batch check with per-job fallback keeps the worker's verdicts;
//  * canAcceptWork() = context idle-capacity and queue bound (index.ts:143-149);
//  * close() rejects buffered and queued jobs with QueueError
//    QUEUE_ERROR_QUEUE_ABORTED (index.ts:193-214, util/queue/errors.ts);
//  * the lodestar_bls_thread_pool_* metrics (metrics/metrics/lodestar.ts:
//    350-430) are kept under their names in `metrics`.
//
// Sets: {type: "single" | "aggregate", pubkey | pubkeys, signingRoot
// (Uint8Array 32), signature (Uint8Array)}.  A pubkey is {index} (a row of
// the HBM index2pubkey table) or {raw: Uint8Array(96)} (uncompressed x||y).
const path = require("path");

const addon = require(path.join(__dirname, "bgv.node"));

const MAX_SIGNATURE_SETS_PER_JOB = 128; // multithread/index.ts:39
const MAX_BUFFERED_SIGS = 32; // multithread/index.ts:48
const MAX_BUFFER_WAIT_MS = 100; // multithread/index.ts:57
const MAX_JOBS_CAN_ACCEPT_WORK = 512; // multithread/index.ts:62
const MAX_SETS_PER_DEVICE_BATCH = 1 << 17;
const RAW_BIT = 0x80000000;
const EMPTY_JOB = -10; // BGV internal code: a job without sets

class QueueError extends Error {
  // util/queue/errors.ts: LodestarError<{code: QueueErrorCode.QUEUE_ABORTED}>
  constructor(code = "QUEUE_ERROR_QUEUE_ABORTED") {
    super(code);
    this.type = {code};
    this.code = code;
  }
}

// multithread/utils.ts:4-19
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
}

// the caller-side checks of getAggregatedPubkey (chain/bls/utils.ts:5-16),
// made before queueing so a bad call cannot fail a batch it shares
function checkSets(sets) {
  for (const s of sets) {
    const pks = s.type === "single" ? [s.pubkey] : s.pubkeys;
    if (!pks || pks.length === 0 || pks.some((pk) => !pk)) throw Error("EMPTY_AGGREGATE_ARRAY");
    for (const pk of pks) if (pk.raw && pk.raw.length !== 96) throw Error("raw pubkeys must be 96-byte uncompressed");
    if (!s.signingRoot || s.signingRoot.length !== 32) throw Error("signingRoot must be 32 bytes");
  }
}

function aggregatedPubkeysCount(sets) {
  let n = 0;
  for (const s of sets) if (s.type === "aggregate") n += s.pubkeys.length;
  return n;
}

// jobs (arrays of sets) -> the SoA batch of include/bgv.h bgv_batch
function encodeJobs(jobs) {
  let n = 0;
  for (const j of jobs) n += j.length;
  const jobOffsets = new Uint32Array(jobs.length + 1);
  const pkOffsets = new Uint32Array(n + 1);
  const idx = [];
  const raw = [];
  const msgs = new Uint8Array(Math.max(n, 1) * 32);
  const sigs = new Uint8Array(Math.max(n, 1) * 192);
  const sigLen = new Uint32Array(Math.max(n, 1));
  let i = 0;
  jobs.forEach((job, k) => {
    for (const s of job) {
      const pks = s.type === "single" ? [s.pubkey] : s.pubkeys;
      if (!pks || pks.length === 0) throw Error("EMPTY_AGGREGATE_ARRAY"); // PublicKey.aggregate, utils.ts:11
      for (const pk of pks) {
        if (pk.raw) {
          idx.push((RAW_BIT | raw.length) >>> 0);
          raw.push(pk.raw);
        } else {
          idx.push(pk.index >>> 0);
        }
      }
      pkOffsets[i + 1] = idx.length;
      msgs.set(s.signingRoot, 32 * i);
      sigLen[i] = s.signature.length;
      if (s.signature.length === 96 || s.signature.length === 192) sigs.set(s.signature, 192 * i);
      i++;
    }
    jobOffsets[k + 1] = i;
  });
  const rawPks = new Uint8Array(Math.max(raw.length, 1) * 96);
  raw.forEach((r, k) => rawPks.set(r, 96 * k));
  return {jobOffsets, pkOffsets, pkIndices: Uint32Array.from(idx.length ? idx : [0]), msgs, sigs, sigLen, rawPks};
}

function jobOutcome(r) {
  if (r === 1) return {ok: true, value: true};
  if (r === 0) return {ok: true, value: false};
  if (r === EMPTY_JOB) return {ok: false, error: Error("Empty signature set")}; // maybeBatch.ts:29-31
  return {ok: false, error: Error(`BLST_ERROR: ${addon.codeName(-r)}`)};
}

function newMetrics() {
  const hist = () => ({count: 0, sum: 0});
  return {
    lodestar_bls_aggregated_pubkeys_total: 0,
    lodestar_bls_thread_pool_time_seconds_sum: 0,
    lodestar_bls_thread_pool_success_jobs_signature_sets_count: 0,
    lodestar_bls_thread_pool_error_jobs_signature_sets_count: 0,
    lodestar_bls_thread_pool_queue_job_wait_time_seconds: hist(),
    lodestar_bls_thread_pool_queue_length: 0,
    lodestar_bls_thread_pool_workers_busy: 0,
    lodestar_bls_thread_pool_job_groups_started_total: 0,
    lodestar_bls_thread_pool_jobs_started_total: 0,
    lodestar_bls_thread_pool_sig_sets_started_total: 0,
    lodestar_bls_thread_pool_batch_retries_total: 0,
    lodestar_bls_thread_pool_batch_sigs_success_total: 0,
    lodestar_bls_thread_pool_latency_to_worker: hist(),
    lodestar_bls_thread_pool_latency_from_worker: hist(),
    lodestar_bls_worker_thread_time_per_sigset_seconds: hist(),
  };
}

function observe(h, v) {
  h.count++;
  h.sum += v;
}

class BlsGpuVerifier {
  constructor({device = 0, maxSetsPerDeviceBatch = MAX_SETS_PER_DEVICE_BATCH} = {}) {
    this.ctx = addon.open(device);
    this.maxSetsPerDeviceBatch = maxSetsPerDeviceBatch;
    this.jobs = [];
    this.bufferedJobs = null;
    this.busy = 0; // device batches in flight (one context = one worker)
    this.closed = false;
    this.metrics = newMetrics();
    this.runJob = this.runJob.bind(this);
    this.runBufferedJobs = this.runBufferedJobs.bind(this);
  }

  // syncPubkeys / addPubkey (pubkeyCache.ts:56-77): 48-byte compressed keys
  syncPubkeys(firstIndex, pubkeys48) {
    addon.pubkeysSet(this.ctx, firstIndex, pubkeys48, 0);
  }

  // multithread/index.ts:143-149 with the context as the only worker
  canAcceptWork() {
    return !this.closed && this.busy < 1 && this.jobs.length < MAX_JOBS_CAN_ACCEPT_WORK;
  }

  async verifySignatureSets(sets, opts = {}) {
    if (this.closed) throw new QueueError();
    checkSets(sets);
    this.metrics.lodestar_bls_aggregated_pubkeys_total += aggregatedPubkeysCount(sets);
    if (opts.verifyOnMainThread) {
      // high priority, unbuffered: one synchronous device batch
      const res = addon.verifySync(this.ctx, encodeJobs([sets]));
      this.recordWork([{sets}], res);
      const o = jobOutcome(res.results[0]);
      if (!o.ok) throw o.error;
      return o.value;
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) => this.queueBlsWork(chunk, opts))
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((r) => r === true);
  }

  // multithread/index.ts:255-292
  queueBlsWork(sets, opts) {
    if (this.closed) return Promise.reject(new QueueError());
    return new Promise((resolve, reject) => {
      const job = {resolve, reject, addedTimeMs: Date.now(), sets};
      if (opts.batchable) {
        if (!this.bufferedJobs) {
          this.bufferedJobs = {jobs: [], sigCount: 0, timeout: setTimeout(this.runBufferedJobs, MAX_BUFFER_WAIT_MS)};
        }
        this.bufferedJobs.jobs.push(job);
        this.bufferedJobs.sigCount += sets.length;
        if (this.bufferedJobs.sigCount > MAX_BUFFERED_SIGS) {
          clearTimeout(this.bufferedJobs.timeout);
          this.runBufferedJobs();
        }
      } else {
        this.jobs.push(job);
        setTimeout(this.runJob, 0);
      }
    });
  }

  // multithread/index.ts:425-431
  runBufferedJobs() {
    if (this.bufferedJobs) {
      this.jobs.push(...this.bufferedJobs.jobs);
      this.bufferedJobs = null;
      setTimeout(this.runJob, 0);
    }
  }

  // every queued job up to maxSetsPerDeviceBatch sets
  prepareWork() {
    const jobs = [];
    let totalSigs = 0;
    while (this.jobs.length > 0 && (jobs.length === 0 || totalSigs + this.jobs[0].sets.length <= this.maxSetsPerDeviceBatch)) {
      const job = this.jobs.shift();
      jobs.push(job);
      totalSigs += job.sets.length;
    }
    return jobs;
  }

  // multithread/index.ts:297-391
  async runJob() {
    if (this.closed || this.busy >= 1) return;
    const jobs = this.prepareWork();
    if (jobs.length === 0) return;
    this.busy++;
    const m = this.metrics;
    try {
      const now = Date.now();
      let started = 0;
      for (const job of jobs) {
        observe(m.lodestar_bls_thread_pool_queue_job_wait_time_seconds, (now - job.addedTimeMs) / 1000);
        started += job.sets.length;
      }
      m.lodestar_bls_thread_pool_job_groups_started_total += 1;
      m.lodestar_bls_thread_pool_jobs_started_total += jobs.length;
      m.lodestar_bls_thread_pool_sig_sets_started_total += started;
      const res = await addon.verify(this.ctx, encodeJobs(jobs.map((j) => j.sets)));
      this.recordWork(jobs, res);
      jobs.forEach((job, k) => {
        const o = jobOutcome(res.results[k]);
        if (o.ok) job.resolve(o.value);
        else job.reject(o.error);
      });
    } catch (e) {
      for (const job of jobs) job.reject(e);
    }
    this.busy--;
    setTimeout(this.runJob, 0);
  }

  recordWork(jobs, res) {
    const m = this.metrics;
    let ok = 0;
    let err = 0;
    jobs.forEach((job, k) => {
      if (res.results[k] >= 0) ok += job.sets.length;
      else err += job.sets.length;
    });
    const workerSec = (res.workerEndMs - res.workerStartMs) / 1000;
    m.lodestar_bls_thread_pool_time_seconds_sum += workerSec;
    if (ok + err > 0) observe(m.lodestar_bls_worker_thread_time_per_sigset_seconds, workerSec / (ok + err));
    m.lodestar_bls_thread_pool_success_jobs_signature_sets_count += ok;
    m.lodestar_bls_thread_pool_error_jobs_signature_sets_count += err;
    m.lodestar_bls_thread_pool_batch_retries_total += res.batchRetries;
    m.lodestar_bls_thread_pool_batch_sigs_success_total += res.batchSigsSuccess;
  }

  // gauges sampled at scrape time (index.ts:135-139)
  metricsSnapshot() {
    this.metrics.lodestar_bls_thread_pool_queue_length = this.jobs.length;
    this.metrics.lodestar_bls_thread_pool_workers_busy = this.busy;
    return this.metrics;
  }

  // multithread/index.ts:193-214
  async close() {
    if (this.closed) return;
    this.closed = true;
    if (this.bufferedJobs) {
      clearTimeout(this.bufferedJobs.timeout);
      for (const job of this.bufferedJobs.jobs) job.reject(new QueueError());
      this.bufferedJobs = null;
    }
    for (const job of this.jobs) job.reject(new QueueError());
    this.jobs = [];
    addon.close(this.ctx); // waits for the batch in flight (the context mutex)
  }
}

module.exports = {
  addon, BlsGpuVerifier, QueueError, chunkifyMaximizeChunkSize, encodeJobs, checkSets,
  MAX_BUFFERED_SIGS, MAX_BUFFER_WAIT_MS, MAX_JOBS_CAN_ACCEPT_WORK,
};
