"use strict";
// IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-51) over
// the N-API addon, in plain CommonJS so it runs on the Node in this image.
// The TypeScript class a maintainer adds (INTEGRATION.md section 4) has the
// same shape; this file is what the addon's tests drive.
//
// Sets: {type: "single" | "aggregate", pubkey | pubkeys, signingRoot
// (Uint8Array 32), signature (Uint8Array)}.  A pubkey is {index} (a row of
// the HBM index2pubkey table) or {raw: Uint8Array(96)} (uncompressed x||y).
const path = require("path");

const addon = require(path.join(__dirname, "bgv.node"));

const MAX_SIGNATURE_SETS_PER_JOB = 128; // multithread/index.ts:39
const RAW_BIT = 0x80000000;
const EMPTY_JOB = -10; // BGV internal code: a job without sets

// multithread/utils.ts:4-19
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
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
  if (r === 1) return true;
  if (r === 0) return false;
  if (r === EMPTY_JOB) throw Error("Empty signature set"); // maybeBatch.ts:29-31
  throw Error(`BLST_ERROR: ${addon.codeName(-r)}`);
}

class BlsGpuVerifier {
  constructor({device = 0} = {}) {
    this.ctx = addon.open(device);
    this.inFlight = 0;
    this.closed = false;
  }

  // syncPubkeys / addPubkey (pubkeyCache.ts:56-77): 48-byte compressed keys
  syncPubkeys(firstIndex, pubkeys48) {
    addon.pubkeysSet(this.ctx, firstIndex, pubkeys48, 0);
  }

  canAcceptWork() {
    return !this.closed && this.inFlight < 4;
  }

  // every chunk of <= 128 sets is one job; all jobs of a call go to the device
  // as ONE batch; the call resolves to the AND of the job verdicts
  async verifySignatureSets(sets, opts = {}) {
    if (this.closed) throw Object.assign(Error("QUEUE_ABORTED"), {code: "QUEUE_ABORTED"});
    const jobs = chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB);
    const batch = encodeJobs(jobs);
    this.inFlight++;
    let res;
    try {
      res = opts.verifyOnMainThread ? addon.verifySync(this.ctx, batch) : await addon.verify(this.ctx, batch);
    } finally {
      this.inFlight--;
    }
    let all = true;
    for (const r of res) all = jobOutcome(r) && all;
    return all;
  }

  async close() {
    if (this.closed) return;
    this.closed = true;
    addon.close(this.ctx);
  }
}

module.exports = {addon, BlsGpuVerifier, chunkifyMaximizeChunkSize, encodeJobs};
