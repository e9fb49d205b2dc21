"use strict";
// Node-level throughput of BlsGpuVerifier under the gossip queues' concurrency
// (network/gossip/validation/queue.ts:14: beacon_attestation maxConcurrency 64, LIFO): C
// concurrent callers each validate one single-set batchable attestation at a time
// (verifySignatureSets([set], {batchable: true}), as validateGossipAttestation does), for
// `seconds`, over one verifier.  Prints one JSON line per buffering setting with sets/s and
// per-call latency percentiles.  backend "cpu": the same callers over CpuPoolVerifier (the
// C++ restatement of the verify path behind BlsMultiThreadWorkerPool's buffering, `workers`
// packages at once) -- the like-for-like CPU row.
//   node gossip_bench.js [seconds=8] [callers=64] [settings="63:1,64:1,32:100,16:1"] [backend=gpu|cpu] [workers=16]
process.env.UV_THREADPOOL_SIZE = process.env.UV_THREADPOOL_SIZE || "32"; // before any async work
const path = require("path");
const crypto = require("crypto");
const {BlsGpuVerifier, addon} = require(path.join(__dirname, "..", "..", "lodestar_amd", "node", "BlsGpuVerifier.js"));

const seconds = Number(process.argv[2] || 8);
const callers = Number(process.argv[3] || 64);
const settings = (process.argv[4] || "63:1,64:1,32:100,16:1").split(",").map((s) => s.split(":").map(Number));
const backend = process.argv[5] || "gpu";
const workers = Number(process.argv[6] || 16);
const NKEYS = 16384;

function pct(xs, p) {
  const s = xs.slice().sort((a, b) => a - b);
  return s[Math.min(s.length - 1, Math.floor(p * s.length))];
}

async function runOne(ctx, sets, maxBufferedSigs, maxBufferWaitMs, secs = seconds, make = null) {
  const v = make ? make() : new BlsGpuVerifier({ctx, maxBufferedSigs, maxBufferWaitMs});
  let next = 0;
  let done = 0;
  let bad = 0;
  const lat = [];
  const t0 = process.hrtime.bigint();
  const deadline = t0 + BigInt(Math.round(secs * 1e9));
  async function caller() {
    while (process.hrtime.bigint() < deadline) {
      const s = sets[next++ % sets.length];
      const a = process.hrtime.bigint();
      const ok = await v.verifySignatureSets([s], {batchable: true});
      lat.push(Number(process.hrtime.bigint() - a) / 1e6);
      if (!ok) bad++;
      done++;
    }
  }
  await Promise.all(Array.from({length: callers}, caller));
  const dt = Number(process.hrtime.bigint() - t0) / 1e9;
  // the verifier shares the context: do not close it here
  if (v.bufferedJobs) clearTimeout(v.bufferedJobs.timeout);
  return {
    maxBufferedSigs,
    maxBufferWaitMs,
    callers,
    sets: done,
    invalid: bad,
    seconds: dt,
    sets_per_s: done / dt,
    latency_ms: {p50: pct(lat, 0.5), p90: pct(lat, 0.9), p99: pct(lat, 0.99)},
  };
}

async function main() {
  const ctx = addon.init([0]);
  const sks = new Uint8Array(32 * NKEYS);
  for (let i = 0; i < NKEYS; i++) {
    const k = crypto.createHash("sha256").update("gossip-key-" + i).digest();
    k[0] &= 0x3f; // < 2^254 < r, nonzero with overwhelming probability
    sks.set(k, 32 * i);
  }
  addon.keygen(ctx, sks, 0);
  const msgs = new Uint8Array(32 * NKEYS);
  for (let i = 0; i < NKEYS; i++) msgs.set(crypto.createHash("sha256").update("gossip-msg-" + i).digest(), 32 * i);
  const sigs = addon.sign(ctx, sks, msgs);
  const sets = [];
  for (let i = 0; i < NKEYS; i++) {
    sets.push({type: "single", pubkey: i, signingRoot: msgs.slice(32 * i, 32 * i + 32), signature: sigs.slice(96 * i, 96 * i + 96)});
  }
  if (backend === "cpu") {
    const {CpuPoolVerifier, loadAddon} = require(path.join(__dirname, "CpuPoolVerifier.js"));
    const cpu = loadAddon();
    const pubkeys96 = cpu.skToPk96(sks);
    const make = () => new CpuPoolVerifier({cpu, pubkeys96, workers});
    await runOne(ctx, sets, 32, 100, 1, make); // warm-up
    const r = await runOne(ctx, sets, 32, 100, seconds, make);
    r.backend = "cpu-port";
    r.workers = workers;
    process.stdout.write(JSON.stringify(r) + "\n");
    addon.close(ctx);
    return;
  }
  await runOne(ctx, sets, 32, 2, 2); // warm-up: first launches load code objects
  for (const [b, w] of settings) {
    const r = await runOne(ctx, sets, b, w);
    r.backend = "gpu";
    process.stdout.write(JSON.stringify(r) + "\n");
  }
  addon.close(ctx);
}

main().catch((e) => {
  process.stderr.write(String(e && e.stack) + "\n");
  process.exit(1);
});
