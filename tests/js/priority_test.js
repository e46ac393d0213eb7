"use strict";
// GPU test of the non-blocking verifyOnMainThread path (lodestar_amd/napi/index.js
// verifyPriority; reference multithread/index.ts:155-167, chain/validation/block.ts:146):
// with a >= 50,000-set bulk batch in flight on the device, a verifyOnMainThread
// single set resolves first, the Node event loop keeps turning (setImmediate
// probe: every gap < 2 ms while the priority call is pending and until the bulk
// batch resolves), and both verdicts are right.  Inputs come from
// tests/test_napi.py (device keys and signatures, written to files).
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const {addon, BlsGpuVerifier, encodeJobs, PRIORITY_CUS} = require(path.join(__dirname, "..", "..", "lodestar_amd", "napi"));
const dir = process.argv[2];
const rd = (name) => new Uint8Array(fs.readFileSync(path.join(dir, name)));
const u32 = (name) => { const b = fs.readFileSync(path.join(dir, name)); return new Uint32Array(b.buffer, b.byteOffset, b.length / 4); };

async function main() {
  const meta = JSON.parse(fs.readFileSync(path.join(dir, "meta.json")));
  const table = rd("table96.bin"), msgs = rd("msgs.bin"), sigs = rd("sigs.bin");
  const pkOff = u32("pk_offsets.bin"), pkIdx = u32("pk_indices.bin");
  const n = meta.n_sets;
  const set = (i) => {
    const pubkeys = [];
    for (let k = pkOff[i]; k < pkOff[i + 1]; k++) pubkeys.push({index: pkIdx[k]});
    return {type: "aggregate", pubkeys, signingRoot: msgs.subarray(32 * i, 32 * i + 32), signature: sigs.subarray(96 * i, 96 * i + 96)};
  };
  const bulkSets = [];
  for (let i = 0; i < n - 1; i++) bulkSets.push(set(i));
  const single = [set(n - 1)];

  const prioCus = process.env.PRIO_CUS === undefined ? PRIORITY_CUS : Number(process.env.PRIO_CUS);
  const verifier = new BlsGpuVerifier({device: 0, priorityCus: prioCus});
  verifier.pubkeysSet(0, table, 1);
  // warm both contexts (first-call allocations are not what is measured) and
  // the JIT: encodeJobs sees a bulk-sized input before the window, so the
  // priority call inside it does not pay a deoptimisation for the new shapes
  assert.strictEqual(await verifier.verifySignatureSets(bulkSets.slice(0, 8192)), true);
  assert.strictEqual(await verifier.verifySignatureSets(single, {verifyOnMainThread: true}), true);
  assert.strictEqual(await verifier.verifySignatureSets(single, {verifyOnMainThread: true}), true);

  const t0 = process.hrtime.bigint();
  const ms = () => Number(process.hrtime.bigint() - t0) / 1e6;
  // the synchronous part of a priority call with the device idle, piece by piece
  const idleIssue = {};
  {
    const a = ms();
    const b = encodeJobs([single]);
    const c = ms();
    const p = addon.verify(verifier.prio, b);
    const d = ms();
    await p;
    const e = ms();
    idleIssue.encode = +(c - a).toFixed(3);
    idleIssue.addon_verify = +(d - c).toFixed(3);
    idleIssue.device = +(e - d).toFixed(3);
  }
  // collect the set-up's garbage before the bulk call, not inside the window
  if (global.gc) global.gc();
  for (let k = 0; k < 4; k++) await new Promise((r) => setImmediate(r));
  let bulkDone = null, prioDone = null, prioStart = null;
  const bulkStart = ms();
  const bulk = verifier.verifySignatureSets(bulkSets).then((v) => { bulkDone = ms(); return v; });
  // wait (event loop free) until the bulk device batch is in flight
  while (verifier.busy === 0) await new Promise((r) => setImmediate(r));
  const inflight = ms();
  // the bulk call's encoding leaves young garbage and new type feedback in
  // verifySignatureSets / checkSets / encodeJobs: a minor collection and one
  // priority call (awaited) take the one-time scavenge and re-optimisation
  // outside the window, as in a node whose priority calls recur every slot
  if (global.gc) global.gc({type: "minor"});
  for (let k = 0; k < 4; k++) await new Promise((r) => setImmediate(r));
  assert.strictEqual(await verifier.verifySignatureSets(single, {verifyOnMainThread: true}), true, "warm priority verdict");
  const warmDone = ms();
  // the window: from the priority call until the bulk batch's device work
  // completes (its result callback and the resolution of its jobs are the
  // pool's own bookkeeping on the main thread, as in the reference)
  let maxGap = 0, last = ms(), probes = 0, resultsAt = null;
  const record = verifier.recordWork.bind(verifier);
  verifier.recordWork = (jobs, res) => {
    if (jobs.length > 1 && resultsAt === null) resultsAt = ms();  // the bulk batch's results reach JS
    record(jobs, res);
  };
  const gaps = [];
  const probe = () => new Promise((resolve) => {
    const tick = () => {
      const t = ms();
      if (t - last > 1.0) gaps.push([+last.toFixed(3), +(t - last).toFixed(3)]);
      if (resultsAt === null || t < resultsAt) maxGap = Math.max(maxGap, t - last);
      last = t;
      probes++;
      if (bulkDone === null) setImmediate(tick); else resolve();
    };
    setImmediate(tick);
  });
  await new Promise((r) => setImmediate(r));
  last = ms();
  const probing = probe();
  prioStart = ms();
  const prio = verifier.verifySignatureSets(single, {verifyOnMainThread: true}).then((v) => { prioDone = ms(); return v; });
  const prioIssued = ms();
  const issueParts = verifier.lastPriorityIssue;
  const [bv, pv] = await Promise.all([bulk, prio]);
  await probing;
  console.log(JSON.stringify({n_bulk: bulkSets.length, bulk_start_ms: bulkStart, bulk_in_flight_ms: inflight, warm_done_ms: warmDone, prio_start_ms: prioStart, prio_issue_ms: prioIssued - prioStart, issue_parts: issueParts, idle_issue: idleIssue,
    prio_done_ms: prioDone, bulk_done_ms: bulkDone, prio_latency_ms: prioDone - prioStart, max_event_loop_gap_ms: maxGap,
    bulk_results_at_ms: resultsAt, probes, gaps_over_1ms: gaps, prio_cus: prioCus}));
  assert.strictEqual(bv, true, "bulk verdict");
  assert.strictEqual(pv, true, "priority verdict");
  assert.ok(prioDone < bulkDone, `priority call resolved after the bulk batch (${prioDone} >= ${bulkDone} ms)`);
  assert.ok(maxGap < 2.0, `event loop blocked for ${maxGap} ms`);
  await verifier.close();
  console.log("priority test OK");
}

main().catch((e) => { console.error(e); process.exit(1); });
