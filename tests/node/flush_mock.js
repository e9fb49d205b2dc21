"use strict";
// BlsGpuVerifier's pubkey queue against a mock addon (no GPU): runs are packed by the hook and
// uploaded in index order; only a run whose records fail to decode is reported and dropped;
// any other failure keeps that run and every later one queued and reaches the caller; the
// flush leaves the event loop free (state-transition/src/cache/epochContext.ts:702-705).
const path = require("path");
const assert = require("assert");
const addonPath = path.join(__dirname, "..", "..", "lodestar_amd", "node", "blsgpu.node");
const puts = [];
let failNext = null;
const mock = {
  init: () => ({}),
  close: () => {},
  strerror: (c) => "code " + c,
  verify: (ctx, jobs) => new Promise((r) => setTimeout(() => r(jobs.map(() => 1)), 3)),
  pubkeysPutAsync: (ctx, first, buf, fmt) =>
    new Promise((resolve, reject) =>
      setTimeout(() => {
        if (failNext !== null) {
          const e = new Error("mock failure " + failNext);
          e.bgvCode = failNext;
          failNext = null;
          return reject(e);
        }
        puts.push([first, Buffer.from(buf)]);
        resolve();
      }, 1)),
};
require.cache[addonPath] = {id: addonPath, filename: addonPath, loaded: true, exports: mock};
const {BlsGpuVerifier} = require(path.join(__dirname, "..", "..", "lodestar_amd", "node", "BlsGpuVerifier.js"));

const key = (i) => {
  const b = new Uint8Array(48);
  b[0] = 0x80 | (i & 0x1f);
  b[45] = i & 0xff;
  b[46] = (i >> 8) & 0xff;
  b[47] = (i >> 16) & 0xff;
  return b;
};

(async () => {
  const v = new BlsGpuVerifier({});
  const hook = v.pubkeyAddedHook();
  // out of order and in two runs: uploaded as [3, 5) then [5, 7), every byte in place
  for (const i of [5, 6, 3, 4]) hook(i, key(i), {});
  await v.flushPubkeys();
  assert.deepStrictEqual(puts.map((p) => [p[0], p[1].length / 48]), [[3, 2], [5, 2]]);
  for (const [first, bytes] of puts)
    for (let k = 0; k < bytes.length / 48; k++)
      assert.deepStrictEqual(new Uint8Array(bytes.subarray(48 * k, 48 * k + 48)), key(first + k));
  // a run longer than PUBKEY_RUN (8192) goes in pieces
  puts.length = 0;
  for (let i = 7; i < 7 + 20000; i++) hook(i, key(i), {});
  await v.flushPubkeys();
  assert.deepStrictEqual(puts.map((p) => [p[0], p[1].length / 48]), [[7, 8192], [8199, 8192], [16391, 3616]]);
  // a device error wrote nothing: the run stays queued with the ones after it, the caller sees it
  puts.length = 0;
  hook(20007, key(20007), {});
  hook(20009, key(20009), {});
  failNext = -30;
  await assert.rejects(v.flushPubkeys(), (e) => e.bgvCode === -30);
  assert.strictEqual(v.pendingRuns.length, 2);
  assert.strictEqual(v.pendingKeys, 2);
  await v.flushPubkeys();
  assert.deepStrictEqual(puts.map((p) => p[0]), [20007, 20009]);
  // undecodable records (a BLST status): committed by the library, reported once and dropped
  const reports = [];
  v.onPubkeyError = (e, first, n) => reports.push([e.bgvCode, first, n]);
  puts.length = 0;
  hook(20010, key(20010), {});
  hook(20012, key(20012), {});
  failNext = -1;
  await v.flushPubkeys();
  assert.deepStrictEqual(reports, [[-1, 20010, 1]]);
  assert.deepStrictEqual(puts.map((p) => p[0]), [20012]);
  assert.strictEqual(v.pendingRuns.length, 0);

  // 65,536 keys queued, then 64 one-set calls: the flush they wait for holds the loop briefly
  const msg = new Uint8Array(32), sig = new Uint8Array(96);
  const one = () => v.verifySignatureSets([{type: "single", pubkey: 0, signingRoot: msg, signature: sig}],
    {batchable: true});
  let worst = 0;
  const bulk = new Uint8Array(48 * 65536);
  for (let rep = 0; rep < 3; rep++) {
    const base = 30000 + rep * 65536;
    for (let i = 0; i < 65536; i++) hook(base + i, bulk.subarray(48 * i, 48 * i + 48), {});
    if (global.gc) global.gc();  // the hook's garbage is the caller's; keep its collection out of the window
    let last = process.hrtime.bigint();
    let maxGap = 0;
    const ticker = setInterval(() => {
      const t = process.hrtime.bigint();
      maxGap = Math.max(maxGap, Number(t - last) / 1e6);
      last = t;
    }, 0);
    const calls = [];
    for (let k = 0; k < 64; k++) calls.push(one());
    assert.ok((await Promise.all(calls)).every((x) => x === true));
    await v.flushPubkeys();
    clearInterval(ticker);
    if (rep) worst = Math.max(worst, maxGap);  // rep 0 includes the JIT's first compilations
  }
  console.log(JSON.stringify({mock_pubkey_flush: {max_event_loop_gap_ms: worst}}));
  assert.ok(worst < 5, `event loop held ${worst} ms by the flush`);
  await v.close();
  console.log("flush mock ok");
})().catch((e) => {
  console.error(e);
  process.exit(1);
});
