"use strict";
// GPU test of the N-API addon (lodestar_amd/napi) from plain JavaScript:
// the golden batch (tests/golden/batch_vectors.json, oracle-generated) through
// addon.verify / addon.verifySync, then the IBlsVerifier wrapper with the
// reference e2e semantics (e2e/chain/bls/multithread.test.ts:8-104).
// Run by tests/test_napi.py on the GPU box; exits non-zero on any mismatch.
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const {addon, BlsGpuVerifier} = require(path.join(__dirname, "..", "..", "lodestar_amd", "napi"));
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

async function main() {
  const v = JSON.parse(fs.readFileSync(path.join(golden, "batch_vectors.json")));
  const interop = JSON.parse(fs.readFileSync(path.join(golden, "interop-pubkeys.json")));
  const pk48 = new Uint8Array(48 * interop.length);
  interop.forEach((p, k) => pk48.set(hex(p), 48 * k));

  const verifier = new BlsGpuVerifier({device: 0});
  verifier.syncPubkeys(0, pk48);
  assert.strictEqual(addon.pubkeysCount(verifier.ctx), interop.length);
  assert.deepStrictEqual(Array.from(addon.pubkeysValidate(verifier.ctx, pk48.slice(0, 48 * 4))), [0, 0, 0, 0]);

  // 1. golden batch, async (libuv pool) and sync paths
  const {batch, expected} = goldenBatch(v);
  const got = await addon.verify(verifier.ctx, batch);
  assert.deepStrictEqual(Array.from(got), expected, "addon.verify vs golden");
  assert.deepStrictEqual(Array.from(addon.verifySync(verifier.ctx, batch)), expected, "addon.verifySync vs golden");
  // several in flight at once on one context (serialised by the addon)
  const many = await Promise.all([0, 1, 2, 3].map(() => addon.verify(verifier.ctx, batch)));
  for (const r of many) assert.deepStrictEqual(Array.from(r), expected);

  // 2. IBlsVerifier semantics (multithread.test.ts:8-104)
  const sets = v.jobs[0].sets.map((s) => ({
    type: "single", pubkey: {raw: hex(v.raw_pubkeys[s.raw])}, signingRoot: hex(s.msg), signature: hex(s.sig),
  }));
  assert.strictEqual(await verifier.verifySignatureSets(sets), true);
  assert.strictEqual(await verifier.verifySignatureSets(sets, {batchable: true}), true);
  assert.strictEqual(await verifier.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
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

  await verifier.close();
  await assert.rejects(verifier.verifySignatureSets(sets), /QUEUE_ABORTED/);
  console.log("addon golden test OK:", Array.from(got).join(","));
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});
