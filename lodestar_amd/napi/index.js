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

// Every context's device batch runs on a libuv pool thread; contexts on
// different devices run concurrently only if the pool has a thread for each
// (default 4).  libuv reads UV_THREADPOOL_SIZE once, when the pool first
// starts: in a host that has already done fs / crypto work (Lodestar has) this
// default is ignored, so the launcher sets it before Node starts
// (INTEGRATION.md section 4) and the constructor warns when it is too small.
const UV_POOL_PRESET = process.env.UV_THREADPOOL_SIZE;
if (!UV_POOL_PRESET) process.env.UV_THREADPOOL_SIZE = "16";

const addon = require(path.join(__dirname, "bgv.node"));

// the library must be compiled from the sources beside it (tools/build.py
// embeds their SHA-256 as bgv_build_id; lodestar_amd/native.py source_hash
// is the same digest): a stale libbgv.so is refused instead of run
function sourceHash(root = path.join(__dirname, "..", "..")) {
  const fs = require("fs");
  const crypto = require("crypto");
  const csrc = path.join(root, "lodestar_amd", "csrc");
  const files = fs.readdirSync(csrc).filter((f) => f.endsWith(".h") || f.endsWith(".hip")).sort()
    .map((f) => "lodestar_amd/csrc/" + f).concat(["include/bgv.h"]);
  const h = crypto.createHash("sha256");
  for (const rel of files) {
    const data = fs.readFileSync(path.join(root, rel));
    const len = Buffer.alloc(8);
    len.writeUInt32LE(data.length % 0x100000000, 0);
    len.writeUInt32LE(Math.floor(data.length / 0x100000000), 4);
    h.update(Buffer.concat([Buffer.from(rel + "\0"), len, data]));
  }
  return h.digest("hex");
}

// an install that ships bgv.node + libbgv.so without the csrc tree cannot be
// compared: the check is skipped with a warning (INTEGRATION.md section 3)
function checkBuildId(id = addon.buildId()) {
  let want;
  try {
    want = sourceHash();
  } catch (e) {
    console.warn(`BlsGpuVerifier: libbgv.so build id not checked (sources not readable: ${e.message})`);
    return;
  }
  if (id !== want && !id.startsWith(want + "+")) {
    throw Error(`libbgv.so was built from other sources (id ${id.slice(0, 16)}, tree ${want.slice(0, 16)}): rebuild`);
  }
}
checkBuildId();

const MAX_SIGNATURE_SETS_PER_JOB = 128; // multithread/index.ts:39
const MAX_BUFFERED_SIGS = 32; // multithread/index.ts:48
const MAX_BUFFER_WAIT_MS = 100; // multithread/index.ts:57
const MAX_JOBS_CAN_ACCEPT_WORK = 512; // multithread/index.ts:62
const MAX_SETS_PER_DEVICE_BATCH = 1 << 17;
const now = () => Number(process.hrtime.bigint()) / 1e6;
// CUs of the first device kept for verifyOnMainThread (bgv_cfg.cu_split): the top 32 ids are one CU of every
// shader engine, and any reservation costs that device's bulk context ~13% at C4 and ~20% at the 8-GPU shard size
// (DESIGN.md §3), so the priority side takes 32 rather than 8.  The default reserves them only on a pool of two or
// more devices, where sharded batches give device 0 a RESERVED_CAP-weighted share; a one-device pool keeps the
// whole chip for its bulk batches unless priorityCus asks for the split.
const PRIORITY_CUS = 32;
const RESERVED_CAP = require("./reserved_cap.json").RESERVED_CAP; // dist.py RESERVED_CAP: bulk pace of a device with reserved CUs
// a device batch of at least this many sets (and >= 2 jobs) is split by job
// over the idle devices (partial Miller products, ONE combined final
// exponentiation); smaller batches run whole on one device while the other
// devices take the next batch (lodestar_amd/verifier.py SHARD_MIN_SETS)
const SHARD_MIN_SETS = 4096;
// device batches in flight per GPU, one context each: the next batches' hash,
// pubkey and decode kernels fill the SIMDs that a batch's one-wave Miller
// phase leaves idle (C4 36.7 -> 33.1 ms per batch with 3, C4/8 shards
// 9.65 -> 8.35 ms; profiles/r06b_overlap_sizes.txt, DESIGN.md §5)
const CONTEXTS_PER_DEVICE = 3;
// non-batchable jobs start once a macro task passes without a new job
// (bounded), so the per-block calls of a range-sync segment
// (verifyBlocksSignatures.ts:30-47, sleep(0) every 8 blocks) coalesce
const MAX_QUIET_WAITS = 8;
const RAW_BIT = 0x80000000;
// the G1 generator, 96-byte uncompressed, and the identity signature: the priority context's sizing job
const G1_GENERATOR_96 = Uint8Array.from(Buffer.from(
  "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb" +
  "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1", "hex"));
const IDENTITY_SIG_96 = (() => { const b = new Uint8Array(96); b[0] = 0xc0; return b; })();
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

// jobs (arrays of sets) -> the SoA batch of include/bgv.h bgv_batch.  Two
// passes (count, then fill typed arrays): a 2^17-set batch allocates its
// arrays once instead of growing JS arrays of up to ~17M indices, which kept
// the main thread in the garbage collector
function encodeJobs(jobs) {
  let n = 0, nIdx = 0, nRaw = 0;
  for (const j of jobs) {
    n += j.length;
    for (const s of j) {
      const pks = s.type === "single" ? [s.pubkey] : s.pubkeys;
      if (!pks || pks.length === 0) throw Error("EMPTY_AGGREGATE_ARRAY"); // PublicKey.aggregate, utils.ts:11
      nIdx += pks.length;
      for (const pk of pks) if (pk.raw) nRaw++;
    }
  }
  const jobOffsets = new Uint32Array(jobs.length + 1);
  const pkOffsets = new Uint32Array(n + 1);
  const pkIndices = new Uint32Array(Math.max(nIdx, 1));
  const rawPks = new Uint8Array(Math.max(nRaw, 1) * 96);
  const msgs = new Uint8Array(Math.max(n, 1) * 32);
  const sigs = new Uint8Array(Math.max(n, 1) * 192);
  const sigLen = new Uint32Array(Math.max(n, 1));
  let i = 0, x = 0, r = 0;
  jobs.forEach((job, k) => {
    for (const s of job) {
      if (s.type === "single") {
        const pk = s.pubkey;
        if (pk.raw) { pkIndices[x++] = (RAW_BIT | r) >>> 0; rawPks.set(pk.raw, 96 * r++); } else pkIndices[x++] = pk.index >>> 0;
      } else {
        for (const pk of s.pubkeys) {
          if (pk.raw) { pkIndices[x++] = (RAW_BIT | r) >>> 0; rawPks.set(pk.raw, 96 * r++); } else pkIndices[x++] = pk.index >>> 0;
        }
      }
      pkOffsets[i + 1] = x;
      msgs.set(s.signingRoot, 32 * i);
      sigLen[i] = s.signature.length;
      if (s.signature.length === 96 || s.signature.length === 192) sigs.set(s.signature, 192 * i);
      i++;
    }
    jobOffsets[k + 1] = i;
  });
  return {jobOffsets, pkOffsets, pkIndices, msgs, sigs, sigLen, rawPks};
}

// device work of a job in Montgomery Fp products (lodestar_amd/dist.py
// job_work, from tools/fpmul_counts.json): per set 13,790, per pubkey
// reference 11 (one G1 mixed addition of the gather)
const WORK_PER_SET = 13790;
const WORK_PER_PUBKEY = 11;
function jobWork(sets) {
  let refs = 0;
  for (const s of sets) refs += s.type === "single" ? 1 : s.pubkeys.length;
  return sets.length * WORK_PER_SET + refs * WORK_PER_PUBKEY;
}

// whole jobs to `world` shards, greedy by work (largest first, each to the
// least loaded shard), job order kept inside a shard (dist.py shard_jobs);
// caps: relative speed per shard (load compared as load / cap)
function shardJobs(weights, world, caps = null) {
  const shards = Array.from({length: world}, () => []);
  const load = new Array(world).fill(0);
  const cap = caps || new Array(world).fill(1);
  let floor = Infinity;
  for (const w of weights) if (w > 0 && w < floor) floor = w;
  if (floor === Infinity) floor = 1;
  const order = weights.map((s, j) => j).sort((a, b) => weights[b] - weights[a] || a - b);
  for (const j of order) {
    let r = 0;
    for (let k = 1; k < world; k++) if (load[k] / cap[k] < load[r] / cap[r]) r = k;
    shards[r].push(j);
    load[r] += Math.max(weights[j], floor);
  }
  return shards.map((s) => s.sort((a, b) => a - b));
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
    // verifyOnMainThread calls (mainThreadDurationInThreadPool, multithread/index.ts:156-167)
    lodestar_bls_thread_pool_main_thread_time_seconds: hist(),
  };
}

function observe(h, v) {
  h.count++;
  h.sum += v;
}

class BlsGpuVerifier {
  // devices: HIP device ordinals, one context each, all owned by this process
  // (chain/chain.ts:199-202 constructs one verifier per node); every context
  // holds a replica of the pubkey table
  // priorityCus: CUs of the first device reserved for verifyOnMainThread
  // (bgv_cfg.cu_split, a multiple of 8): a priority context runs there, the
  // bulk context of that device leaves them free (~13-20% of its throughput
  // whatever the count: the shader engines that lost a CU set the pace;
  // sharded batches give that device a RESERVED_CAP-weighted shard).  Default:
  // PRIORITY_CUS on a pool of two or more devices, 0 on one device (the
  // priority context then shares every CU)
  // blsVerifyAllMultiThread (chain/options.ts:14, multithread/index.ts:124): verifyOnMainThread
  // calls join the pool's queue like any other; no CUs are then reserved and
  // no priority context is opened
  // contextsPerDevice: device batches in flight per GPU (one context each,
  // each with its own table replica); a batch large enough to shard is split
  // over one idle context per device
  constructor({device = 0, devices = null, maxSetsPerDeviceBatch = MAX_SETS_PER_DEVICE_BATCH, shardMinSets = SHARD_MIN_SETS,
    priorityCus = null, blsVerifyAllMultiThread = false, contextsPerDevice = CONTEXTS_PER_DEVICE} = {}) {
    const ids = devices && devices.length ? devices : [device];
    if (!(contextsPerDevice >= 1)) throw new Error(`contextsPerDevice ${contextsPerDevice}`);
    if (priorityCus === null || priorityCus === undefined) priorityCus = ids.length > 1 ? PRIORITY_CUS : 0;
    if (blsVerifyAllMultiThread) priorityCus = 0;
    this.blsVerifyAllMultiThread = blsVerifyAllMultiThread;
    // every device batch holds a libuv pool thread (napi_async_work); the pool
    // size is read once, when the pool first starts, so the launcher must set
    // UV_THREADPOOL_SIZE before Node runs any async work (INTEGRATION.md 4)
    // UV_THREADPOOL_SIZE; judged on the value the process started with: the
    // 16 this module assigns when it was unset only counts if the pool had
    // not started yet, which the module cannot tell, so it assumes libuv's 4
    const pool = Number(UV_POOL_PRESET) || 4;
    const nCtx = ids.length * contextsPerDevice;
    if (nCtx + 2 > pool) {
      const was = UV_POOL_PRESET ? `UV_THREADPOOL_SIZE=${pool}` : "UV_THREADPOOL_SIZE unset at start (libuv default 4)";
      console.warn(`BlsGpuVerifier: ${nCtx} device contexts with ${was}: device batches may ` +
        "serialise and starve other pool work; start Node with UV_THREADPOOL_SIZE >= contexts + 2");
    }
    // context k runs on device entry ctxDev[k]; every bulk context of the first
    // device leaves the reserved CUs free (one unmasked context would put bulk
    // waves on them)
    this.ctxDev = [];
    this.ctxs = [];
    ids.forEach((d, i) => {
      for (let c = 0; c < contextsPerDevice; c++) {
        this.ctxs.push(addon.open(d, i === 0 && priorityCus > 0 ? -priorityCus : 0));
        this.ctxDev.push(i);
      }
    });
    this.nDevices = ids.length;
    this.contextsPerDevice = contextsPerDevice;
    this.ctx = this.ctxs[0];
    // verifyOnMainThread's own context (with its own table replica and mutex):
    // it never waits for a bulk batch's context lock or, with priorityCus, its
    // waves.  Under blsVerifyAllMultiThread nothing uses it: the blocking
    // verifySignatureSetsSync then runs on the first bulk context
    this.prio = blsVerifyAllMultiThread ? null : addon.open(ids[0], priorityCus > 0 ? priorityCus : 0);
    this.prioReserved = priorityCus > 0;
    this.priorityCus = priorityCus;
    if (this.prio) this.warmPriority();
    this.prioBusy = 0;
    this.idle = this.ctxs.map(() => true);
    this.maxSetsPerDeviceBatch = maxSetsPerDeviceBatch;
    this.shardMinSets = shardMinSets;
    this.jobs = [];
    this.queuedSets = 0;
    this.bufferedJobs = null;
    this.busy = 0; // device batches in flight
    this.closed = false;
    this.runScheduled = false;
    this.pushSeq = 0;
    this.seenSeq = 0;
    this.quietWaits = 0;
    this.metrics = newMetrics();
    this.runJob = this.runJob.bind(this);
    this.runBufferedJobs = this.runBufferedJobs.bind(this);
  }

  // syncPubkeys / addPubkey (pubkeyCache.ts:56-77): 48-byte compressed keys, every replica
  syncPubkeys(firstIndex, pubkeys48) {
    this.pubkeysSet(firstIndex, pubkeys48, 0);
  }

  // rows in either format (0: 48-byte compressed, 1: 96-byte uncompressed) into every replica
  pubkeysSet(firstIndex, bytes, format) {
    for (const c of this.allContexts()) addon.pubkeysSet(c, firstIndex, bytes, format);
  }

  // sizes the priority context's work buffers for a full job (128 sets) at
  // construction, so a verifyOnMainThread call never frees and regrows them
  // (a hipFree synchronises the device: it would wait for the bulk contexts'
  // batches in flight).  One dummy job: the generator as a raw key and the
  // identity signature; its verdict is ignored.
  warmPriority() {
    const set = {type: "single", pubkey: {raw: G1_GENERATOR_96}, signingRoot: new Uint8Array(32), signature: IDENTITY_SIG_96};
    addon.verifySync(this.prio, encodeJobs([new Array(MAX_SIGNATURE_SETS_PER_JOB).fill(set)]));
  }

  allContexts() {
    return this.prio ? this.ctxs.concat([this.prio]) : this.ctxs.slice();
  }

  // multithread/index.ts:143-149.  A queued job joins the next device batch,
  // so work is accepted while fewer than MAX_JOBS_CAN_ACCEPT_WORK jobs and
  // less than one full device batch of sets are queued, batch in flight or
  // not (gating on idle devices would stop the network processor,
  // network/processor/index.ts:406, for every 5-40 ms device batch)
  canAcceptWork() {
    return !this.closed && this.jobs.length < MAX_JOBS_CAN_ACCEPT_WORK && this.queuedSets < this.maxSetsPerDeviceBatch;
  }

  async verifySignatureSets(sets, opts = {}) {
    if (this.closed) throw new QueueError();
    checkSets(sets);
    this.metrics.lodestar_bls_aggregated_pubkeys_total += aggregatedPubkeysCount(sets);
    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) return this.verifyPriority(sets);
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) => this.queueBlsWork(chunk, opts))
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((r) => r === true);
  }

  // verifyOnMainThread (multithread/index.ts:155-167; chain/validation/block.ts:146
  // for a gossip block's proposer signature): high priority and unbuffered, as
  // the reference runs it at once on the main thread, but without blocking the
  // event loop: one device batch on the priority context, on the libuv pool.
  // It bypasses the buffer, the job queue and the bulk contexts' locks.
  async verifyPriority(sets) {
    this.prioBusy++;
    const t0 = now();
    try {
      const batch = encodeJobs([sets]);
      const t1 = now();
      const pending = addon.verify(this.prio, batch);
      this.lastPriorityIssue = {encodeMs: t1 - t0, queueMs: now() - t1};
      const res = await pending;
      this.recordWork([{sets}], res);
      const o = jobOutcome(res.results[0]);
      if (!o.ok) throw o.error;
      return o.value;
    } finally {
      // timed in a finally like the reference's mainThreadDurationInThreadPool
      // (multithread/index.ts:156-167): calls that throw are observed too
      observe(this.metrics.lodestar_bls_thread_pool_main_thread_time_seconds, (now() - t0) / 1e3);
      this.prioBusy--;
    }
  }

  // BlsSingleThreadVerifier.verifySignatureSets (singleThread.ts:14-35):
  // maybeBatch on the calling thread, for callers that want exactly that;
  // the pool's verifyOnMainThread uses verifyPriority instead
  verifySignatureSetsSync(sets) {
    if (this.closed) throw new QueueError();
    checkSets(sets);
    const res = addon.verifySync(this.prio || this.ctx, encodeJobs([sets]));
    this.recordWork([{sets}], res);
    const o = jobOutcome(res.results[0]);
    if (!o.ok) throw o.error;
    return o.value;
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
        this.pushJobs([job]);
        this.pushSeq++;
        this.scheduleRun();
      }
    });
  }

  pushJobs(jobs) {
    for (const j of jobs) this.queuedSets += j.sets.length;
    this.jobs.push(...jobs);
  }

  // the first look comes a macro task later, as in the reference
  // (setTimeout(runJob, 0), multithread/index.ts:242,299); the quiet-window
  // re-looks use setImmediate, which Node does not clamp to 1 ms, so a lone
  // block-import job pays microseconds for the coalescing, not milliseconds
  scheduleRun(quiet = false) {
    if (!this.runScheduled) {
      this.runScheduled = true;
      if (quiet) setImmediate(this.runJob);
      else setTimeout(this.runJob, 0);
    }
  }

  // multithread/index.ts:425-431 (the buffer has already waited: no quiet window)
  runBufferedJobs() {
    if (this.bufferedJobs) {
      this.pushJobs(this.bufferedJobs.jobs);
      this.bufferedJobs = null;
      this.scheduleRun();
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
    this.queuedSets -= totalSigs;
    return jobs;
  }

  // idle contexts: the first idle one of each device (spread, for sharding)
  // and the idle one on the least busy device (for a whole batch)
  idleContexts() {
    const busyOn = new Array(this.nDevices).fill(0);
    this.idle.forEach((f, k) => { if (!f) busyOn[this.ctxDev[k]]++; });
    const spread = [];
    const seen = new Set();
    let best = -1;
    this.idle.forEach((f, k) => {
      if (!f) return;
      const dv = this.ctxDev[k];
      if (!seen.has(dv)) { seen.add(dv); spread.push(k); }
      if (best < 0 || busyOn[dv] < busyOn[this.ctxDev[best]]) best = k;
    });
    return {spread, best};
  }

  // multithread/index.ts:297-391: every idle context takes a device batch; a
  // batch of >= shardMinSets sets is split over one idle context per device
  runJob() {
    this.runScheduled = false;
    while (!this.closed && this.jobs.length > 0) {
      const {spread: idle, best} = this.idleContexts();
      if (idle.length === 0) return; // a finishing batch reschedules
      if (this.pushSeq !== this.seenSeq && this.quietWaits < MAX_QUIET_WAITS) {
        // jobs arrived since the last look: wait one more macro task
        this.seenSeq = this.pushSeq;
        this.quietWaits++;
        this.scheduleRun(true);
        return;
      }
      this.quietWaits = 0;
      this.seenSeq = this.pushSeq;
      const jobs = this.prepareWork();
      let n = 0;
      for (const j of jobs) n += j.sets.length;
      const devs = idle.length > 1 && jobs.length > 1 && n >= this.shardMinSets ? idle : [best];
      for (const k of devs) this.idle[k] = false;
      this.runDeviceBatch(jobs, devs);
    }
  }

  async runDeviceBatch(jobs, devs) {
    this.busy++;
    this.peakBusy = Math.max(this.peakBusy || 0, this.busy); // device batches in flight at once (test hook)
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
      const res = devs.length === 1
        ? await addon.verify(this.ctxs[devs[0]], encodeJobs(jobs.map((j) => j.sets)))
        : await this.verifySharded(jobs.map((j) => j.sets), devs);
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
    for (const k of devs) this.idle[k] = true;
    this.scheduleRun();
  }

  // SURVEY 8e: jobs sharded by work (sets + pubkey references) over the devices, one partial Miller
  // product per shard (bgv_partial, concurrently on the libuv pool), ONE final
  // exponentiation of their product (bgv_combine_final); only when it fails
  // does each shard localise its failing jobs (bgv_partial_finish, the
  // worker's per-job retry).  Returns the result shape of addon.verify.
  async verifySharded(jobSets, devs) {
    // the first device's bulk context leaves CUs to the priority context and
    // runs at RESERVED_CAP of the others' pace (dist.py)
    const caps = devs.map((k) => (this.ctxDev[k] === 0 && this.prioReserved ? RESERVED_CAP : 1));
    const shards = shardJobs(jobSets.map(jobWork), devs.length, caps);
    const live = [];
    shards.forEach((ids, r) => ids.length && live.push({ctx: this.ctxs[devs[r]], ids}));
    if (live.length === 1) return addon.verify(live[0].ctx, encodeJobs(jobSets));
    const parts = await Promise.all(live.map((s) => addon.partial(s.ctx, encodeJobs(s.ids.map((k) => jobSets[k])))));
    const millers = new Uint8Array(576 * live.length);
    parts.forEach((p, k) => millers.set(p.miller, 576 * k));
    const valid = await addon.combineFinal(live[0].ctx, millers);
    // a verifyOnMainThread call that ran on a context in between replaced its
    // pending partial (bgv error -7): that shard is verified again from scratch
    const finals = valid ? parts : await Promise.all(live.map((s) => addon.partialFinish(s.ctx).catch((e) => {
      if (!/bgv error -7/.test(e.message)) throw e;
      return addon.verify(s.ctx, encodeJobs(s.ids.map((k) => jobSets[k])));
    })));
    const results = new Int32Array(jobSets.length);
    let sigsOk = 0;
    live.forEach((s, k) => s.ids.forEach((j, i) => {
      results[j] = finals[k].results[i];
      if (valid && results[j] === 1) sigsOk += jobSets[j].length;
    }));
    return {
      results, batchRetries: valid ? 0 : 1, batchSigsSuccess: sigsOk,
      pubkeysAggregated: parts.reduce((a, p) => a + p.pubkeysAggregated, 0),
      deviceMs: Math.max(...parts.map((p) => p.deviceMs)),
      workerStartMs: Math.min(...parts.map((p) => p.workerStartMs)),
      workerEndMs: Math.max(...finals.map((p) => p.workerEndMs)),
      shards: live.length,
    };
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
    this.metrics.lodestar_bls_thread_pool_workers_busy = this.idle.filter((f) => !f).length;
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
    this.queuedSets = 0;
    for (const c of this.allContexts()) addon.close(c); // each waits for its batch in flight (the context mutex)
  }
}

// BlsSingleThreadVerifier (chain/bls/singleThread.ts:7-46), which chain.ts:200-202
// builds instead of the pool when blsVerifyAllMainThread is set: maybeBatch on
// one device context, blocking the calling thread as blst does on the main
// thread (addon.verifySync); canAcceptWork is always true.  Its pubkey table
// is its own replica.
class BlsGpuSingleThreadVerifier {
  constructor({device = 0} = {}) {
    this.ctx = addon.open(device, 0);
    this.closed = false;
    this.metrics = {lodestar_bls_aggregated_pubkeys_total: 0, lodestar_bls_thread_pool_main_thread_time_seconds: {count: 0, sum: 0}};
  }

  syncPubkeys(firstIndex, pubkeys48) {
    addon.pubkeysSet(this.ctx, firstIndex, pubkeys48, 0);
  }

  pubkeysSet(firstIndex, bytes, format) {
    addon.pubkeysSet(this.ctx, firstIndex, bytes, format);
  }

  async verifySignatureSets(sets) {
    if (this.closed) throw new QueueError();
    this.metrics.lodestar_bls_aggregated_pubkeys_total += aggregatedPubkeysCount(sets);
    checkSets(sets); // getAggregatedPubkey's checks (utils.ts:5-16)
    const t0 = now();
    const res = addon.verifySync(this.ctx, encodeJobs([sets]));
    const o = jobOutcome(res.results[0]);
    if (!o.ok) throw o.error; // only runs without exceptions are timed, as in the reference
    observe(this.metrics.lodestar_bls_thread_pool_main_thread_time_seconds, (now() - t0) / 1e3);
    return o.value;
  }

  async close() {
    if (this.closed) return;
    this.closed = true;
    addon.close(this.ctx);
  }

  canAcceptWork() {
    return true;
  }
}

module.exports = {
  addon, BlsGpuVerifier, BlsGpuSingleThreadVerifier, QueueError, sourceHash, checkBuildId, chunkifyMaximizeChunkSize, encodeJobs, checkSets, shardJobs, jobWork,
  MAX_BUFFERED_SIGS, MAX_BUFFER_WAIT_MS, MAX_JOBS_CAN_ACCEPT_WORK, SHARD_MIN_SETS, PRIORITY_CUS, RESERVED_CAP, CONTEXTS_PER_DEVICE,
};
