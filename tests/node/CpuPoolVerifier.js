"use strict";
// The CPU row of the Node gossip bench -- TEST INFRASTRUCTURE.  IBlsVerifier over the C++
// restatement of the verify path (oracle/cpu/libblscpu.so through tests/node/blscpu.node), with
// BlsMultiThreadWorkerPool's job flow (packages/beacon-node/src/chain/bls/multithread/index.ts):
//   * batchable jobs are buffered; the buffer goes to the job queue when it holds more than
//     MAX_BUFFERED_SIGS (32) sets or MAX_BUFFER_WAIT_MS (100 ms) after its first job (index.ts:258-275);
//   * other jobs go to the queue at once (index.ts:280-283);
//   * an idle worker takes queued jobs up to MAX_SIGNATURE_SETS_PER_JOB (128) sets
//     (prepareWork, index.ts:386-401) and verifies them as one package: batchable jobs in
//     chunks with per-job retry, others alone (worker.ts; blscpu_verify mode 0).
// A worker here is one blscpu_verify call on a libuv pool thread (one thread each), so `workers`
// packages run at once, like Lodestar's worker threads; UV_THREADPOOL_SIZE must be at least
// `workers` (set before the first async call).
// Sets: {type: "single", pubkey: index, signingRoot, signature}; pubkeys index a table of
// 96-byte uncompressed affine keys (the index2pubkey cache).
const fs = require("fs");
const path = require("path");

const MAX_BUFFERED_SIGS = 32;
const MAX_BUFFER_WAIT_MS = 100;
const MAX_SIGNATURE_SETS_PER_JOB = 128;

function loadAddon() {
  const cpu = require(path.join(__dirname, "blscpu.node"));
  const c = fs.readFileSync(path.join(__dirname, "blscpu_consts.bin"));
  const rc = cpu.init(new Uint8Array(c.buffer, c.byteOffset, 288), new Uint8Array(c.buffer, c.byteOffset + 288, 1440));
  if (rc !== 0) throw new Error("blscpu.init failed");
  return cpu;
}

class CpuPoolVerifier {
  constructor({cpu, pubkeys96, workers = 16}) {
    this.cpu = cpu;
    this.pubkeys96 = pubkeys96;
    this.workers = Array.from({length: workers}, () => ({busy: false}));
    this.jobs = [];
    this.bufferedJobs = null;
    this.seed = 1;
  }

  verifySignatureSets(sets, opts = {}) {
    return new Promise((resolve, reject) => {
      const job = {resolve, reject, sets, batchable: Boolean(opts.batchable)};
      if (job.batchable) {
        if (!this.bufferedJobs) {
          this.bufferedJobs = {jobs: [], sigCount: 0, timeout: setTimeout(() => this.runBufferedJobs(), MAX_BUFFER_WAIT_MS)};
        }
        this.bufferedJobs.jobs.push(job);
        this.bufferedJobs.sigCount += sets.length;
        if (this.bufferedJobs.sigCount > MAX_BUFFERED_SIGS) {
          clearTimeout(this.bufferedJobs.timeout);
          this.runBufferedJobs();
        }
      } else {
        this.jobs.push(job);
        setTimeout(() => this.runJob(), 0);
      }
    });
  }

  runBufferedJobs() {
    if (this.bufferedJobs) {
      this.jobs.push(...this.bufferedJobs.jobs);
      this.bufferedJobs = null;
      setTimeout(() => this.runJob(), 0);
    }
  }

  prepareWork() {
    const jobs = [];
    let total = 0;
    while (total < MAX_SIGNATURE_SETS_PER_JOB) {
      const job = this.jobs.shift();
      if (!job) break;
      jobs.push(job);
      total += job.sets.length;
    }
    return jobs;
  }

  async runJob() {
    const worker = this.workers.find((w) => !w.busy);
    if (!worker) return;
    const jobs = this.prepareWork();
    if (jobs.length === 0) return;
    worker.busy = true;
    let n = 0;
    for (const j of jobs) n += j.sets.length;
    const pk = new Uint8Array(96 * n);
    const msgs = new Uint8Array(32 * n);
    const sigs = new Uint8Array(96 * n);
    const lens = new Uint32Array(n);
    const jobs3 = new Uint32Array(3 * jobs.length);
    let s = 0;
    jobs.forEach((j, k) => {
      jobs3[3 * k] = s;
      jobs3[3 * k + 1] = j.sets.length;
      jobs3[3 * k + 2] = j.batchable ? 1 : 0;
      for (const set of j.sets) {
        pk.set(this.pubkeys96.subarray(96 * set.pubkey, 96 * set.pubkey + 96), 96 * s);
        msgs.set(set.signingRoot, 32 * s);
        sigs.set(set.signature.subarray(0, 96), 96 * s);
        lens[s] = set.signature.length;
        s++;
      }
    });
    try {
      const out = await this.cpu.verifyAsync(pk, msgs, sigs, lens, jobs3, 0, 1, this.seed++);
      jobs.forEach((j, k) => j.resolve(out[k] === 1));
    } catch (e) {
      for (const j of jobs) j.reject(e);
    }
    worker.busy = false;
    setTimeout(() => this.runJob(), 0);
  }
}

module.exports = {CpuPoolVerifier, loadAddon};
