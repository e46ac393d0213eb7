"use strict";
// GPU test of the N-API addon (lodestar_amd/napi) from plain JavaScript:
// the golden batch (tests/golden/batch_vectors.json, oracle-generated) through
// addon.verify / addon.verifySync, then the IBlsVerifier wrapper with the
// reference e2e semantics (e2e/chain/bls/multithread.test.ts:8-104).
// Run by tests/test_napi.py on the GPU box; exits non-zero on any mismatch.
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const {addon, BlsGpuVerifier, BlsGpuSingleThreadVerifier, QueueError} = require(path.join(__dirname, "..", "..", "lodestar_amd", "napi"));
const golden = path.join(__dirname, "..", "golden");
const hex = (s) => Uint8Array.from(Buffer.from(s.replace(/^0x/, ""), "hex"));

function goldenBatch(v) {
  const raw = v.raw_pubkeys.map(hex);
  const jobOffsets = [0], pkOffsets = [0], idx = [], msgs = [], sigs = [], sigLen = [], expected = [];
  for (const j of v.jobs) {
    for (const s of j.sets) {
      if (s.raw !== null) idx.push((0x80000000 | s.raw) >>> 0);
      else idx.push(...s.pk);
      pkOffsets.push(idx.length);
      msgs.push(hex(s.msg));
      const sig = hex(s.sig);
      sigLen.push(sig.length);
      const padded = new Uint8Array(192);
      if (sig.length === 96 || sig.length === 192) padded.set(sig);
      sigs.push(padded);
    }
    jobOffsets.push(msgs.length);
    expected.push(j.expected);
  }
  const cat = (arrs, w) => {
    const out = new Uint8Array(Math.max(arrs.length, 1) * w);
    arrs.forEach((a, k) => out.set(a, k * w));
    return out;
  };
  return {
    batch: {
      jobOffsets: Uint32Array.from(jobOffsets), pkOffsets: Uint32Array.from(pkOffsets),
      pkIndices: Uint32Array.from(idx.length ? idx : [0]), msgs: cat(msgs, 32), sigs: cat(sigs, 192),
      sigLen: Uint32Array.from(sigLen.length ? sigLen : [0]), rawPks: cat(raw, 96),
    },
    expected,
  };
}

// the golden jobs as arrays of IBlsVerifier sets (raw pubkeys or table indices)
function goldenJobSets(v) {
  return v.jobs.map((j) => j.sets.map((s) => {
    const sig = hex(s.sig);
    const pks = s.raw !== null ? [{raw: hex(v.raw_pubkeys[s.raw])}] : s.pk.map((i) => ({index: i}));
    return {type: "aggregate", pubkeys: pks, signingRoot: hex(s.msg), signature: sig};
  }));
}

async function main() {
  const v = JSON.parse(fs.readFileSync(path.join(golden, "batch_vectors.json")));
  const interop = JSON.parse(fs.readFileSync(path.join(golden, "interop-pubkeys.json")));
  const pk48 = new Uint8Array(48 * interop.length);
  interop.forEach((p, k) => pk48.set(hex(p), 48 * k));

  const verifier = new BlsGpuVerifier({device: 0});
  assert.strictEqual(verifier.prioReserved, false, "one device: no CU reservation by default");
  verifier.syncPubkeys(0, pk48);
  const extra = new Uint8Array(96 * v.extra_table.length);
  v.extra_table.forEach((p, k) => extra.set(hex(p), 96 * k));
  verifier.pubkeysSet(v.extra_table_base, extra, 1);
  assert.strictEqual(addon.pubkeysCount(verifier.ctx), interop.length + v.extra_table.length);
  assert.strictEqual(addon.pubkeysCount(verifier.prio), interop.length + v.extra_table.length);
  assert.deepStrictEqual(Array.from(addon.pubkeysValidate(verifier.ctx, pk48.slice(0, 48 * 4))), [0, 0, 0, 0]);
  // a gap in the table and an undecodable key are refused
  assert.throws(() => addon.pubkeysSet(verifier.ctx, 5000, pk48.slice(0, 48), 0), /bgv error -4/);
  const badKey = pk48.slice(0, 48);
  badKey[0] &= 0x7f;
  assert.throws(() => addon.pubkeysSet(verifier.ctx, 102, badKey, 0), /BLST_BAD_ENCODING/);

  // 1. golden batch, async (libuv pool) and sync paths
  const {batch, expected} = goldenBatch(v);
  const got = await addon.verify(verifier.ctx, batch);
  assert.deepStrictEqual(Array.from(got.results), expected, "addon.verify vs golden");
  assert.strictEqual(got.batchRetries, 1);
  assert.ok(got.deviceMs > 0 && got.workerEndMs >= got.workerStartMs);
  assert.deepStrictEqual(Array.from(addon.verifySync(verifier.ctx, batch).results), expected, "addon.verifySync vs golden");
  // several in flight at once on one context (serialised by the addon)
  const many = await Promise.all([0, 1, 2, 3].map(() => addon.verify(verifier.ctx, batch)));
  for (const r of many) assert.deepStrictEqual(Array.from(r.results), expected);
  // pkIndices shorter than pkOffsets[n] is refused before any work is queued
  assert.throws(() => addon.verify(verifier.ctx, {...batch, pkIndices: batch.pkIndices.slice(0, 3)}), /pkIndices shorter/);

  // 2. IBlsVerifier semantics (multithread.test.ts:8-104)
  const sets = v.jobs[0].sets.map((s) => ({
    type: "single", pubkey: {raw: hex(v.raw_pubkeys[s.raw])}, signingRoot: hex(s.msg), signature: hex(s.sig),
  }));
  assert.strictEqual(await verifier.verifySignatureSets(sets), true);
  assert.strictEqual(await verifier.verifySignatureSets(sets, {batchable: true}), true);
  const groups0 = verifier.metrics.lodestar_bls_thread_pool_job_groups_started_total;
  assert.strictEqual(await verifier.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
  assert.strictEqual(verifier.metrics.lodestar_bls_thread_pool_job_groups_started_total, groups0, "priority path skips the queue");
  assert.ok(verifier.metrics.lodestar_bls_thread_pool_main_thread_time_seconds.count >= 1, "main-thread duration series");
  const mt0 = verifier.metrics.lodestar_bls_thread_pool_main_thread_time_seconds.count;
  await assert.rejects(verifier.verifySignatureSets([{...sets[0], signature: new Uint8Array(32)}], {verifyOnMainThread: true}),
    /BLST_INVALID_SIZE/);
  assert.strictEqual(verifier.metrics.lodestar_bls_thread_pool_main_thread_time_seconds.count, mt0 + 1, "a throwing call is timed");
  assert.strictEqual(verifier.verifySignatureSetsSync(sets), true);  // BlsSingleThreadVerifier semantics
  const wrongMsg = sets.map((s, k) => (k === 1 ? {...s, signingRoot: hex(v.jobs[0].sets[0].msg).map((b) => b ^ 1)} : s));
  assert.strictEqual(await verifier.verifySignatureSets(wrongMsg), false);
  await assert.rejects(verifier.verifySignatureSets([{...sets[0], signature: new Uint8Array(32)}]), /BLST_INVALID_SIZE/);
  await assert.rejects(verifier.verifySignatureSets([]), /Empty signature set/);
  await assert.rejects(
    verifier.verifySignatureSets([{type: "aggregate", pubkeys: [], signingRoot: new Uint8Array(32), signature: new Uint8Array(96)}]),
    /EMPTY_AGGREGATE_ARRAY/,
  );
  // an aggregate over table indices (golden job 1: k = 5)
  const agg = v.jobs[1].sets.map((s) => ({
    type: "aggregate", pubkeys: s.pk.map((i) => ({index: i})), signingRoot: hex(s.msg), signature: hex(s.sig),
  }));
  assert.strictEqual(await verifier.verifySignatureSets(agg), v.jobs[1].expected === 1);

  // 3. pool scheduling (multithread/index.ts:143-149, 255-431)
  const m = verifier.metrics;
  assert.strictEqual(verifier.canAcceptWork(), true);
  // two batchable calls inside 100 ms are buffered and run as ONE device batch of two jobs
  let groups = m.lodestar_bls_thread_pool_job_groups_started_total;
  let jobsStarted = m.lodestar_bls_thread_pool_jobs_started_total;
  let waits = m.lodestar_bls_thread_pool_queue_job_wait_time_seconds;
  let w0 = {...waits};
  const t0 = Date.now();
  const [b1, b2] = await Promise.all([verifier.verifySignatureSets(sets, {batchable: true}), verifier.verifySignatureSets(sets, {batchable: true})]);
  assert.ok(b1 && b2);
  assert.strictEqual(m.lodestar_bls_thread_pool_job_groups_started_total - groups, 1);
  assert.strictEqual(m.lodestar_bls_thread_pool_jobs_started_total - jobsStarted, 2);
  assert.ok(Date.now() - t0 >= 95, "buffered for the 100 ms window");
  assert.ok((waits.sum - w0.sum) / (waits.count - w0.count) >= 0.09, "queue wait covers the buffer window");
  // more than 32 buffered sigs flush at once
  const many33 = [];
  for (let k = 0; k < 11; k++) many33.push(...sets);
  groups = m.lodestar_bls_thread_pool_job_groups_started_total;
  w0 = {...waits};
  assert.strictEqual(await verifier.verifySignatureSets(many33, {batchable: true}), true);
  assert.strictEqual(m.lodestar_bls_thread_pool_job_groups_started_total - groups, 1);
  assert.ok((waits.sum - w0.sum) / (waits.count - w0.count) < 0.09, "a > 32-sig buffer does not wait for the timer");
  // metrics: retries on a failing batch, sets counted, aggregated keys
  const retries = m.lodestar_bls_thread_pool_batch_retries_total;
  assert.strictEqual(await verifier.verifySignatureSets(wrongMsg), false);
  assert.strictEqual(m.lodestar_bls_thread_pool_batch_retries_total - retries, 1);
  assert.ok(m.lodestar_bls_thread_pool_batch_sigs_success_total > 0);
  assert.ok(m.lodestar_bls_thread_pool_success_jobs_signature_sets_count > 0);
  assert.ok(m.lodestar_bls_thread_pool_error_jobs_signature_sets_count >= 1);
  assert.strictEqual(m.lodestar_bls_aggregated_pubkeys_total, 5 + 1);  // the k=5 aggregate (+ the empty one)
  assert.strictEqual(verifier.metricsSnapshot().lodestar_bls_thread_pool_queue_length, 0);

  // 4. range-sync call pattern (verifyBlocksSignatures.ts:30-47): one
  // non-batchable call per block, sleep(0) after every 8 blocks; the quiet
  // window coalesces the segment's blocks into at most two device batches
  const sleep0 = () => new Promise((r) => setTimeout(r, 0));
  groups = m.lodestar_bls_thread_pool_job_groups_started_total;
  const blockPromises = [];
  for (let i = 0; i < 32; i++) {
    blockPromises.push(verifier.verifySignatureSets(i === 19 ? wrongMsg : sets));
    if ((i + 1) % 8 === 0) await sleep0();
  }
  const blockRes = await Promise.all(blockPromises);
  const cs2Batches = m.lodestar_bls_thread_pool_job_groups_started_total - groups;
  assert.deepStrictEqual(blockRes.map((r, i) => r === (i !== 19)), new Array(32).fill(true));
  assert.ok(cs2Batches <= 2, `32 per-block calls took ${cs2Batches} device batches`);
  console.log(`range-sync pattern: 32 per-block calls -> ${cs2Batches} device batch(es)`);
  // a lone non-batchable job (block import) is dispatched after the
  // reference's one macro task (setTimeout 0, >= 1 ms) plus one unclamped
  // setImmediate look for followers, not after extra 1-ms timer turns
  const loneWaits = [];
  for (let r = 0; r < 5; r++) {
    const w1 = {...waits};
    assert.strictEqual(await verifier.verifySignatureSets(sets), true);
    loneWaits.push((waits.sum - w1.sum) * 1000);
  }
  loneWaits.sort((a, b) => a - b);
  assert.ok(loneWaits[2] <= 3, `lone job waited ${loneWaits[2]} ms before dispatch (median of 5)`);
  console.log(`lone non-batchable job: dispatch wait median ${loneWaits[2]} ms`);

  // 5. back-pressure: queued work joins the next batch, so canAcceptWork stays
  // true while a batch is in flight and turns false once a full next batch
  // (maxSetsPerDeviceBatch sets) is queued
  const small = new BlsGpuVerifier({device: 0, maxSetsPerDeviceBatch: 2 * sets.length});
  small.syncPubkeys(0, pk48);
  const inflight = small.verifySignatureSets(sets);
  await sleep0();
  await sleep0();
  assert.strictEqual(small.canAcceptWork(), true, "accepts while a batch is in flight");
  const q1 = small.verifySignatureSets(sets);
  const q2 = small.verifySignatureSets(sets);
  assert.strictEqual(small.canAcceptWork(), false, "a full next batch is queued");
  assert.deepStrictEqual(await Promise.all([inflight, q1, q2]), [true, true, true]);
  assert.strictEqual(small.canAcceptWork(), true);
  await small.close();

  // 5a. device batches in flight: calls that arrive while a batch runs go to
  // another context of the same GPU at once (contextsPerDevice, default 3)
  const inf = new BlsGpuVerifier({device: 0});
  assert.strictEqual(inf.ctxs.length, 3);
  inf.syncPubkeys(0, pk48);
  const fa = Promise.all(Array.from({length: 16}, () => inf.verifySignatureSets(sets)));
  await sleep0();
  await sleep0();
  const fb = inf.verifySignatureSets(wrongMsg);
  await sleep0();
  await sleep0();
  const fc = inf.verifySignatureSets(sets);
  assert.deepStrictEqual(await Promise.all([fa, fb, fc]), [new Array(16).fill(true), false, true]);
  assert.ok(inf.peakBusy >= 2, `batches in flight at once: ${inf.peakBusy}`);
  await inf.close();

  // 5b. blsVerifyAllMultiThread (chain/options.ts:14): verifyOnMainThread calls
  // join the queue like any other, and no CUs are reserved
  const allMt = new BlsGpuVerifier({device: 0, blsVerifyAllMultiThread: true});
  allMt.syncPubkeys(0, pk48);
  assert.strictEqual(allMt.prioReserved, false);
  assert.strictEqual(allMt.prio, null, "no priority context is opened");
  assert.strictEqual(allMt.verifySignatureSetsSync(sets), true, "the blocking path runs on the bulk context");
  const g0 = allMt.metrics.lodestar_bls_thread_pool_job_groups_started_total;
  assert.strictEqual(await allMt.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
  assert.ok(allMt.metrics.lodestar_bls_thread_pool_job_groups_started_total > g0, "queued like any other call");
  assert.strictEqual(await allMt.verifySignatureSets(wrongMsg, {verifyOnMainThread: true}), false);
  await allMt.close();

  // 5c. BlsSingleThreadVerifier (blsVerifyAllMainThread, chain.ts:200-202)
  const single = new BlsGpuSingleThreadVerifier({device: 0});
  single.syncPubkeys(0, pk48);
  assert.strictEqual(single.canAcceptWork(), true);
  assert.strictEqual(await single.verifySignatureSets(sets), true);
  assert.strictEqual(await single.verifySignatureSets(wrongMsg), false);
  await assert.rejects(single.verifySignatureSets([]), /Empty signature set/);
  assert.strictEqual(single.metrics.lodestar_bls_thread_pool_main_thread_time_seconds.count, 2);
  await single.close();
  await assert.rejects(single.verifySignatureSets(sets), QueueError);

  // 6. several devices owned by one process (SURVEY 8e): two contexts (both on
  // GPU 0 here) verify one batch split by job; partial Miller products, ONE
  // combined final exponentiation; a failing shard is localised per job
  const multi = new BlsGpuVerifier({devices: [0, 0], shardMinSets: 1});
  assert.strictEqual(multi.prioReserved, true, "two devices: device 0 reserves CUs for verifyOnMainThread by default");
  multi.syncPubkeys(0, pk48);
  multi.pubkeysSet(v.extra_table_base, extra, 1);
  const jobSets = v.jobs.map((j) => j.sets);
  // one context of each device entry (contexts 0 .. contextsPerDevice - 1 are the first device's)
  assert.strictEqual(multi.ctxs.length, 2 * multi.contextsPerDevice);
  const two = [0, multi.contextsPerDevice];
  assert.deepStrictEqual(multi.idleContexts().spread, two);
  const mres = await multi.verifySharded(goldenJobSets(v), two);
  assert.strictEqual(mres.shards, 2);
  assert.deepStrictEqual(Array.from(mres.results), expected, "sharded golden batch (faulted shards) vs golden");
  assert.deepStrictEqual(Array.from(mres.results), Array.from(got.results), "sharded == bgv_verify");
  assert.strictEqual(mres.batchRetries, 1);
  const clean = v.jobs.map((j, k) => k).filter((k) => v.jobs[k].expected === 1);
  const cres = await multi.verifySharded(clean.map((k) => goldenJobSets(v)[k]), two);
  assert.deepStrictEqual(Array.from(cres.results), clean.map(() => 1), "sharded clean batch");
  assert.strictEqual(cres.batchRetries, 0);
  // and through the pool: 32 block-sized calls split over both contexts
  const before = multi.metrics.lodestar_bls_thread_pool_job_groups_started_total;
  const segRes = await Promise.all(Array.from({length: 8}, (_, i) => multi.verifySignatureSets(i === 5 ? wrongMsg : sets)));
  assert.deepStrictEqual(segRes, segRes.map((_, i) => i !== 5));
  assert.ok(multi.metrics.lodestar_bls_thread_pool_job_groups_started_total - before >= 1);
  void jobSets;
  await multi.close();

  // 7. close(): buffered and queued jobs reject with QueueError QUEUE_ABORTED
  const pending = verifier.verifySignatureSets(sets, {batchable: true});
  await verifier.close();
  await assert.rejects(pending, (e) => e instanceof QueueError && e.type.code === "QUEUE_ERROR_QUEUE_ABORTED");
  await assert.rejects(verifier.verifySignatureSets(sets), /QUEUE_ERROR_QUEUE_ABORTED/);
  assert.strictEqual(verifier.canAcceptWork(), false);
  console.log("addon golden test OK:", Array.from(got.results).join(","));
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});
