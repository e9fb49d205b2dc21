"use strict";
// Node-side e2e of BlsGpuVerifier, the cases of the reference's
// beacon-node/test/e2e/chain/bls/multithread.test.ts:22-118 run against the MI355X library.
// Usage: node tests/node/multithread_e2e.js [cpu]   (cpu: load/export checks only, no device)
const assert = require("assert");
const path = require("path");
const {BlsGpuVerifier, SignatureSetType, QueueError, chunkifyMaximizeChunkSize, addon, toNativeSet: toNative} = require(
  path.join(__dirname, "..", "..", "lodestar_amd", "node", "BlsGpuVerifier.js")
);

function cpuChecks() {
  for (const f of ["init", "close", "strerror", "pubkeysPut", "keygen", "sign", "verify", "aggregatePubkeys",
    "hashToG2", "pubkeysValidate", "aggregateSignatures", "depositsVerify"]) {
    assert.strictEqual(typeof addon[f], "function", f);
  }
  assert.strictEqual(addon.strerror(8), "BLST_INVALID_SIZE");
  assert.strictEqual(addon.strerror(32), "QUEUE_ABORTED");
  // multithread/utils.test.ts cases of chunkifyMaximizeChunkSize
  const arr = (n) => Array.from({length: n}, (_, i) => i);
  const shape = (n, m) => chunkifyMaximizeChunkSize(arr(n), m).map((c) => c.length);
  assert.deepStrictEqual(shape(0, 128), [0]);
  assert.deepStrictEqual(shape(1, 128), [1]);
  assert.deepStrictEqual(shape(256, 128), [128, 128]);
  assert.deepStrictEqual(shape(257, 128), [129, 128]);
  assert.deepStrictEqual(shape(10, 3), [4, 4, 2]);
  return {cpu: "ok", deviceCount: addon.deviceCount};
}

async function gpuChecks() {
  const N = 3;
  const sks = new Uint8Array(32 * N);
  const msgs = new Uint8Array(32 * N);
  for (let i = 0; i < N; i++) {
    sks.fill(i + 1, 32 * i, 32 * (i + 1)); // SecretKey.fromBytes(Buffer.alloc(32, i + 1))
    msgs.fill(i + 1, 32 * i, 32 * (i + 1));
  }
  const newPool = () => {
    const pool = new BlsGpuVerifier({maxBufferWaitMs: 20});
    addon.keygen(pool.ctx, sks, 0); // pubkeys cached at validator indices 0..N-1
    return pool;
  };
  let pool = newPool();
  const sigs = addon.sign(pool.ctx, sks, msgs);
  const sets = [];
  for (let i = 0; i < N; i++) {
    sets.push({
      type: SignatureSetType.single,
      pubkey: i,
      signingRoot: msgs.slice(32 * i, 32 * (i + 1)),
      signature: sigs.slice(96 * i, 96 * (i + 1)),
    });
  }
  const report = {};
  async function many(sleep, opts) {
    const ps = [];
    for (let i = 0; i < 8; i++) {
      ps.push(pool.verifySignatureSets(sets, opts));
      if (sleep) await new Promise((r) => setTimeout(r, 5));
    }
    const res = await Promise.all(ps);
    res.forEach((v, i) => assert.strictEqual(v, true, `sig set ${i} returned invalid`));
  }
  await many(false, undefined);
  report.sync = "ok";
  await many(true, undefined);
  report.async = "ok";
  await many(true, {batchable: true});
  report.batched = "ok";

  // batched, first is invalid: only its own promise rejects (multithread.test.ts:94-117)
  const invalidSet = Object.assign({}, sets[0], {signature: new Uint8Array(32)});
  const bad = pool.verifySignatureSets([invalidSet], {batchable: true});
  const good = [];
  for (let i = 0; i < 8; i++) good.push(pool.verifySignatureSets(sets, {batchable: true}));
  await assert.rejects(bad, /BLST_INVALID_SIZE/);
  (await Promise.all(good)).forEach((v) => assert.strictEqual(v, true));
  report.firstInvalid = "ok";

  // a wrong signature is false, not an error; mixed batch retried per job
  const wrong = Object.assign({}, sets[0], {signature: sets[1].signature});
  const w = pool.verifySignatureSets([wrong], {batchable: true});
  const g2 = pool.verifySignatureSets(sets, {batchable: true});
  assert.strictEqual(await w, false);
  assert.strictEqual(await g2, true);
  report.wrongSig = "ok";

  // aggregate set: N signers of one message; the aggregate signature is the signature of
  // sum(sk) mod r, the pubkey aggregate is summed from the device cache
  const R = BigInt("0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001");
  let skSum = 0n;
  for (let i = 0; i < N; i++) skSum += BigInt("0x" + Buffer.from(sks.slice(32 * i, 32 * (i + 1))).toString("hex"));
  const skAgg = Uint8Array.from(Buffer.from((skSum % R).toString(16).padStart(64, "0"), "hex"));
  const root = new Uint8Array(32).fill(7);
  const aggSig = addon.sign(pool.ctx, skAgg, root);
  const aggSet = {type: SignatureSetType.aggregate, pubkeys: [0, 1, 2], signingRoot: root, signature: aggSig};
  assert.strictEqual(await pool.verifySignatureSets([aggSet, ...sets], {batchable: true}), true);
  const aggWrong = Object.assign({}, aggSet, {pubkeys: [0, 1]});
  assert.strictEqual(await pool.verifySignatureSets([aggWrong]), false);
  await assert.rejects(pool.verifySignatureSets([Object.assign({}, aggSet, {pubkeys: []})]), /EMPTY_AGGREGATE/);
  report.aggregate = "ok";
  // verifyOnMainThread path and a large call chunked into 128-set jobs
  assert.strictEqual(await pool.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
  const big = [];
  for (let i = 0; i < 300; i++) big.push(sets[i % N]);
  assert.strictEqual(await pool.verifySignatureSets(big, {batchable: true}), true);
  report.chunked = "ok";

  // golden vectors (tests/golden, oracle-signed) with pubkeys passed as 96-B bytes, not indices
  const gold = (f) => JSON.parse(require("fs").readFileSync(path.join(__dirname, "..", "golden", f)));
  const keys = gold("keys.json");
  const hex = (h) => Uint8Array.from(Buffer.from(h, "hex"));
  const gsets = gold("signatures.json").cases.slice(0, 8).map((c) => ({
    type: SignatureSetType.single,
    pubkey: hex(keys.pk_uncompressed[c.key]),
    signingRoot: hex(c.msg),
    signature: hex(c.sig),
  }));
  assert.strictEqual(await pool.verifySignatureSets(gsets, {batchable: true}), true);
  const gswap = [Object.assign({}, gsets[0], {signature: gsets[1].signature})];
  assert.strictEqual(await pool.verifySignatureSets(gswap, {batchable: true}), false);
  report.goldenBytes = "ok";

  // parity hooks through the addon: PublicKey.aggregate (utils.ts:5-16) and hash_to_G2 bytes.
  // Interop keys are appended at cache indices N.. (the cache has no holes), after the keygen keys.
  const K0 = N;
  const pkRec = new Uint8Array(96 * keys.pk_uncompressed.length);
  keys.pk_uncompressed.forEach((h, i) => pkRec.set(hex(h), 96 * i));
  addon.pubkeysPut(pool.ctx, K0, pkRec, 96);
  for (const c of gold("aggregates.json").cases) {
    const idx = Uint32Array.from(c.indices, (i) => i + K0);
    assert.strictEqual(Buffer.from(addon.aggregatePubkeys(pool.ctx, idx)).toString("hex"), c.uncompressed);
  }
  for (const c of gold("hash_to_g2.json").cases.slice(0, 8)) {
    assert.strictEqual(Buffer.from(addon.hashToG2(pool.ctx, hex(c.msg))).toString("hex"), c.uncompressed);
  }
  report.parityHooks = "ok";

  // SURVEY 8(f): deposit key validation, op-pool signature aggregation, deposit signatures
  // against tests/golden/next.json (codes are BLST numbers; 0 = valid)
  const next = gold("next.json");
  const codeName = (c) => (c === 0 ? null : addon.strerror(c));
  assert.deepStrictEqual(pool.validatePubkeys(next.pubkeys.map((c) => hex(c.pk))), next.pubkeys.map((c) => codeName(c.expect)));
  for (const c of next.aggregates) {
    const sigs = c.sigs.map(hex);
    if (c.expect === 0) {
      assert.strictEqual(Buffer.from(pool.aggregateSignatures(sigs)).toString("hex"), c.aggregate);
    } else {
      assert.throws(() => pool.aggregateSignatures(sigs), (e) => e.message === addon.strerror(c.expect));
    }
  }
  const deps = next.deposits.map((c) => ({pubkey: hex(c.pk), signingRoot: hex(c.msg), signature: hex(c.sig)}));
  assert.deepStrictEqual(pool.verifyDeposits(deps), next.deposits.map((c) => c.expect === 1));
  report.next = "ok";

  // metrics parity: the pool's bls / blsThreadPool series (metrics/lodestar.ts:405-494)
  const rec = {};
  const series = (name) => {
    rec[name] = {n: 0, sum: 0, labels: []};
    return {
      inc: (a, b) => {
        const v = typeof a === "object" ? b : a === undefined ? 1 : a;
        if (typeof a === "object") rec[name].labels.push(a);
        rec[name].n++;
        rec[name].sum += v;
      },
      observe: (v) => {
        rec[name].n++;
        rec[name].sum += v;
      },
      set: (v) => (rec[name].sum = v),
      addCollect: (fn) => (rec[name].collect = fn),
      startTimer: () => () => rec[name].n++,
    };
  };
  const names = ["queueLength", "mainThreadDurationInThreadPool", "jobWaitTime", "totalJobsGroupsStarted",
    "totalJobsStarted", "totalSigSetsStarted", "timePerSigSet", "jobsWorkerTime", "successJobsSignatureSetsCount",
    "errorJobsSignatureSetsCount", "batchRetries", "batchSigsSuccess"];
  const metrics = {bls: {aggregatedPubkeys: series("aggregatedPubkeys")}, blsThreadPool: {}};
  for (const n of names) metrics.blsThreadPool[n] = series(n);
  const mpool = new BlsGpuVerifier({maxBufferWaitMs: 20, ctx: pool.ctx}, {metrics});
  const mres = await Promise.all([
    mpool.verifySignatureSets(sets, {batchable: true}),
    mpool.verifySignatureSets([wrong], {batchable: true}),
    mpool.verifySignatureSets([aggSet], {batchable: true}),
    mpool.verifySignatureSets([invalidSet], {batchable: true}).catch((e) => e.message),
  ]);
  assert.deepStrictEqual(mres, [true, false, true, "BLST_INVALID_SIZE"]);
  assert.strictEqual(await mpool.verifySignatureSets(sets, {verifyOnMainThread: true}), true);
  const tp = (n) => rec[n];
  assert.strictEqual(rec.aggregatedPubkeys.sum, 3);
  assert.strictEqual(tp("totalJobsStarted").sum, 4);
  assert.strictEqual(tp("totalSigSetsStarted").sum, N + 3);
  assert.strictEqual(tp("jobWaitTime").n, 4);
  assert.strictEqual(tp("successJobsSignatureSetsCount").sum, N + 2);
  assert.strictEqual(tp("errorJobsSignatureSetsCount").sum, 1);
  assert.ok(tp("batchRetries").sum >= 1, "the mixed batch was retried");
  assert.ok(tp("jobsWorkerTime").sum > 0 && tp("jobsWorkerTime").labels[0].workerId === 0);
  assert.strictEqual(tp("mainThreadDurationInThreadPool").n, 1);
  assert.strictEqual(typeof tp("queueLength").collect, "function");
  report.metrics = "ok";

  // close(): queued work rejects with QUEUE_ABORTED, later calls too (index.ts:176-197,239-241)
  const pending = pool.verifySignatureSets(sets, {batchable: true});
  await pool.close();
  await assert.rejects(pending, (e) => e instanceof QueueError && e.type.code === "QUEUE_ABORTED");
  await assert.rejects(pool.verifySignatureSets(sets), (e) => e instanceof QueueError);
  await pool.close(); // idempotent
  // close() while device calls are in flight (ADVICE r01: the context must outlive them):
  // calls already handed to the library complete with their verdicts, later ones reject,
  // a second close is a no-op, and addon entry points on the closed ctx throw QUEUE_ABORTED
  const pool2 = newPool();
  const inflight = [];
  for (let i = 0; i < 16; i++) inflight.push(addon.verify(pool2.ctx, [{sets: sets.map(toNative), batchable: true}], 0));
  const ctx2 = pool2.ctx;
  await pool2.close();
  await pool2.close();
  const codes = await Promise.all(inflight);
  for (const c of codes) assert.deepStrictEqual(Array.from(c), [1]);
  await assert.rejects(addon.verify(ctx2, [{sets: sets.map(toNative), batchable: true}], 0), /QUEUE_ABORTED/);
  assert.throws(() => addon.aggregatePubkeys(ctx2, Uint32Array.from([0])), /QUEUE_ABORTED/);
  assert.throws(() => addon.hashToG2(ctx2, new Uint8Array(32)), /QUEUE_ABORTED/);
  addon.close(ctx2);
  report.close = "ok";
  return report;
}

(async () => {
  const cpu = cpuChecks();
  const out = process.argv[2] === "cpu" ? cpu : Object.assign(cpu, await gpuChecks());
  console.log(JSON.stringify(out));
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
