"use strict";
/**
 * BlsGpuVerifier — IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-46) on MI355X.
 *
 * Drop-in beside BlsMultiThreadWorkerPool (chain/bls/multithread/index.ts:98-424): the same
 * verifySignatureSets(sets, opts) -> Promise<boolean> and close() -> Promise<void>, the same
 * batchable buffering (index.ts:238-285, 406-412), 128-set jobs (index.ts:39,155-166) and
 * QUEUE_ABORTED after close (index.ts:176-197, 239-241).  Per-job verification, batching and
 * retry run on the GPU (libblsgpu, BGV_MODE_WORKER), so every job's verdict matches the worker's.
 *
 * Pubkeys are validator indices into the device-resident cache (SURVEY §7 "pubkey identity at
 * the boundary", option (a)): set.pubkey / set.pubkeys hold numbers (or {index}).
 *
 * Metrics: with modules.metrics (the beacon node's IMetrics) the verifier feeds the same
 * bls / blsThreadPool series as the pool (metrics/metrics/lodestar.ts:405-494, updated at
 * multithread/index.ts:129-130,136-151,317-367); the whole device is worker 0, and the
 * per-call device time stands in for the worker job time.  latencyToWorker/FromWorker
 * (structured-clone messaging) have no GPU counterpart and are not observed.
 */
const path = require("path");
const addon = require(path.join(__dirname, "blsgpu.node"));

const MAX_SIGNATURE_SETS_PER_JOB = 128; // index.ts:39
// Batchable buffering (index.ts:48,57 use 32 sets / 100 ms for CPU workers).  Gossip caps
// concurrency per topic (64 for attestations, network/gossip/validation/queue.ts:14), so the
// Node-level rate is concurrency / per-call latency: a long buffer wait only adds latency,
// and the library already merges the calls in flight into super-batches.  The flush test is
// the reference's `sigCount > maxBufferedSigs`, so 63 sends the buffer the moment a full
// queue's 64 sets are in it; at 64 every batch waited for the timer.  Measured with 64
// concurrent one-set callers on one MI355X (tests/node/gossip_bench.js,
// profiles/r03/gossip/flush_at_callers.jsonl): 63 / 1 ms 11.6k sets/s at p50 5.4 ms,
// 64 / 1 ms 9.9k at 6.4 ms, 32 / 100 ms 6.2k at 10.3 ms (14.2k at 4.4 ms for 63 / 1 ms with
// the later device chain, profiles/r03/gossip/two_wave_miller.jsonl).
const MAX_BUFFERED_SIGS = 63;
const MAX_BUFFER_WAIT_MS = 1;

const SignatureSetType = {single: "single", aggregate: "aggregate"};
const PUBKEY_RUN = 8192;
// include/blsgpu.h: BGV_BLST_* decode statuses are 1..19 (library codes start at 20)
const isBlstDecodeCode = (code) => typeof code === "number" && code <= -1 && code >= -19;

// One contiguous run of queued validator keys: indices [first, first + n), their 48-byte
// encodings packed in order into bytes (capacity doubles up to PUBKEY_RUN keys).
class PubkeyRun {
  constructor(first) {
    this.first = first;
    this.n = 0;
    this.bytes = new Uint8Array(48 * 64);
  }
  push(pubkey) {
    if (48 * (this.n + 1) > this.bytes.length) {
      const b = new Uint8Array(Math.min(2 * this.bytes.length, 48 * PUBKEY_RUN));
      b.set(this.bytes.subarray(0, 48 * this.n));
      this.bytes = b;
    }
    this.bytes.set(pubkey, 48 * this.n);
    this.n++;
  }
}

class QueueError extends Error {
  constructor(code) {
    super(code);
    this.type = {code};
  }
}

/** chain/bls/multithread/utils.ts:4-19 */
function chunkifyMaximizeChunkSize(arr, minPerChunk) {
  const chunkCount = Math.floor(arr.length / minPerChunk);
  if (chunkCount <= 1) return [arr];
  const perChunk = Math.ceil(arr.length / chunkCount);
  const out = [];
  for (let i = 0; i < arr.length; i += perChunk) out.push(arr.slice(i, i + perChunk));
  return out;
}

/** chain/bls/utils.ts:18-26 */
function getAggregatedPubkeysCount(sets) {
  let n = 0;
  for (const s of sets) if (s.type === SignatureSetType.aggregate) n += s.pubkeys.length;
  return n;
}

function indexOf(pk) {
  return typeof pk === "number" ? pk : pk.index;
}

// A pubkey is a validator index (a number, or a PublicKey tagged with .index by the
// Index2PubkeyCache, INTEGRATION.md), else its 96-B uncompressed bytes (pk.toBytes(false)
// for @chainsafe/bls keys outside the cache, e.g. deposits).
function uncompressed(pk) {
  if (pk instanceof Uint8Array) return pk;
  return pk.toBytes(false);
}

function toNativeSet(s) {
  let pks;
  if (s.type === SignatureSetType.single) pks = [s.pubkey];
  else if (s.type === SignatureSetType.aggregate) pks = s.pubkeys;
  else throw Error("Unknown signature set type");
  if (pks.every((pk) => indexOf(pk) !== undefined)) {
    return {pkIndices: Uint32Array.from(pks, indexOf), msg: s.signingRoot, sig: s.signature};
  }
  const bytes = new Uint8Array(96 * pks.length);
  pks.forEach((pk, i) => bytes.set(uncompressed(pk), 96 * i));
  return {pkBytes: bytes, msg: s.signingRoot, sig: s.signature};
}

class BlsGpuVerifier {
  constructor(opts = {}, modules = {}) {
    this.metrics = modules.metrics || null;
    this.ctx = opts.ctx || addon.init(opts.devices || []);
    this.pendingRuns = []; // PubkeyRun in hook order
    this.pendingKeys = 0;
    this.flushing = null;
    this.onPubkeyError = opts.onPubkeyError || null;
    this.blsVerifyAllMultiThread = opts.blsVerifyAllMultiThread || false;
    this.maxBufferedSigs = opts.maxBufferedSigs || MAX_BUFFERED_SIGS;
    this.maxBufferWaitMs = opts.maxBufferWaitMs || MAX_BUFFER_WAIT_MS;
    this.jobs = [];
    this.bufferedJobs = null;
    this.closed = false;
    this.counters = {aggregatedPubkeys: 0, batchRetries: 0, successJobsSignatureSetsCount: 0, errorJobsSignatureSetsCount: 0};
    const metrics = this.metrics;
    if (metrics) {
      metrics.blsThreadPool.queueLength.addCollect(() => metrics.blsThreadPool.queueLength.set(this.jobs.length));
    }
  }

  /**
   * Index2PubkeyCache growth -> device cache (INTEGRATION.md §2): a function for
   * state-transition's pubkey-added hook, called with (index, 48-byte pubkey, PublicKey).  It
   * tags the PublicKey with .index (so sets built by the reference's producers travel as
   * indices) and queues the key; queued keys go to the device in contiguous runs before the
   * next verification or every 65,536 keys, off the event loop (flushPubkeys).
   */
  pubkeyAddedHook() {
    return (index, pubkey, pk) => {
      if (pk && typeof pk === "object") pk.index = index;
      // packed into its run here, in the caller's time (the state transition adds keys one at a
      // time), so a flush hands whole runs to the addon without touching each key again
      let r = this.pendingRuns[this.pendingRuns.length - 1];
      if (!r || r.first + r.n !== index || r.n >= PUBKEY_RUN) {
        r = new PubkeyRun(index);
        this.pendingRuns.push(r);
      }
      r.push(pubkey);
      this.pendingKeys++;
      // a gap error here reappears at the next verifySignatureSets, which awaits the flush
      if (this.pendingKeys >= 65536) this.flushPubkeys().catch(() => {});
    };
  }

  /**
   * Uploads the queued keys in contiguous runs with the addon's asynchronous put (a libuv pool
   * thread decodes them; the library publishes a run once every device holds it, without
   * waiting for running verifies), so a validator-set growth never stalls the event loop
   * (EpochContext.addPubkey, state-transition/src/cache/epochContext.ts:702-705;
   * pubkeyCache.ts:56-77).  One flush chain at a time; keys queued meanwhile join it.
   * Only a run whose records fail to decode (a BLST status) is committed -- with those indices
   * marked, so sets naming them reject BGV_E_BAD_INDEX -- then reported once (onPubkeyError,
   * else a console warning) and dropped, so one bad key cannot stop later uploads or
   * verification.  Any other failure (a gap in the indices, a device or memory error) wrote
   * nothing: that run stays queued with every run after it, and the error reaches the caller.
   * The runs are packed as the hook receives the keys, so the event loop only sorts a few run
   * records here and hands the addon views of their bytes (the addon holds a reference to each
   * until its put completes).
   */
  flushPubkeys() {
    if (this.closed) return Promise.resolve();
    if (!this.flushing && this.pendingRuns.length) {
      this.flushing = this._flushRuns().finally(() => {
        this.flushing = null;
      });
    }
    return this.flushing || Promise.resolve();
  }

  async _flushRuns() {
    while (this.pendingRuns.length && !this.closed) {
      const runs = this.pendingRuns;
      this.pendingRuns = [];
      this.pendingKeys = 0;
      let sorted = true;
      for (let k = 1; k < runs.length && sorted; k++) sorted = runs[k].first > runs[k - 1].first;
      if (!sorted) runs.sort((a, b) => a.first - b.first);
      let i = 0;
      try {
        for (; i < runs.length; i++) {
          const r = runs[i];
          try {
            await addon.pubkeysPutAsync(this.ctx, r.first, r.bytes.subarray(0, 48 * r.n), 48);
          } catch (e) {
            if (!isBlstDecodeCode(e.bgvCode) || this.closed) throw e;
            this.reportPubkeyError(e, r.first, r.n);
          }
        }
      } finally {
        if (i < runs.length) {
          this.pendingRuns = runs.slice(i).concat(this.pendingRuns);
          this.pendingKeys = this.pendingRuns.reduce((a, r) => a + r.n, 0);
        }
      }
    }
  }

  reportPubkeyError(e, first, n) {
    const msg = `BlsGpuVerifier: pubkeys [${first}, ${first + n}) uploaded with undecodable keys marked: ${e.message}`;
    if (this.onPubkeyError) this.onPubkeyError(e, first, n);
    else console.warn(msg);
  }

  async verifySignatureSets(sets, opts = {}) {
    if (this.pendingRuns.length || this.flushing) await this.flushPubkeys();
    const nAgg = getAggregatedPubkeysCount(sets);
    this.counters.aggregatedPubkeys += nAgg;
    if (this.metrics) this.metrics.bls.aggregatedPubkeys.inc(nAgg);
    if (opts.verifyOnMainThread && !this.blsVerifyAllMultiThread) {
      // index.ts:138-151: one job verified at once (no buffering)
      const timer = this.metrics ? this.metrics.blsThreadPool.mainThreadDurationInThreadPool.startTimer() : null;
      try {
        const codes = await addon.verify(this.ctx, [{sets: sets.map(toNativeSet), batchable: false}], 1);
        return unwrap(codes[0]);
      } finally {
        if (timer) timer();
      }
    }
    const results = await Promise.all(
      chunkifyMaximizeChunkSize(sets, MAX_SIGNATURE_SETS_PER_JOB).map((chunk) =>
        this.queueBlsWork({opts, sets: chunk.map(toNativeSet)})
      )
    );
    if (results.length === 0) throw Error("Empty results array");
    return results.every((v) => v === true);
  }

  // index.ts:176-197.  Idempotent; device calls already in flight complete (the library
  // drains them before releasing the context), queued and later jobs reject QUEUE_ABORTED.
  async close() {
    if (this.closed) return;
    if (this.bufferedJobs) clearTimeout(this.bufferedJobs.timeout);
    const pending = this.jobs.concat(this.bufferedJobs ? this.bufferedJobs.jobs : []);
    for (const job of pending) job.reject(new QueueError("QUEUE_ABORTED"));
    this.jobs = [];
    this.bufferedJobs = null;
    this.closed = true;
    addon.close(this.ctx);
  }

  queueBlsWork(workReq) {
    if (this.closed) return Promise.reject(new QueueError("QUEUE_ABORTED"));
    return new Promise((resolve, reject) => {
      const job = {resolve, reject, workReq, addedTimeMs: Date.now()};
      if (workReq.opts.batchable) {
        if (!this.bufferedJobs) {
          this.bufferedJobs = {jobs: [], sigCount: 0, timeout: setTimeout(this.runBufferedJobs, this.maxBufferWaitMs)};
        }
        this.bufferedJobs.jobs.push(job);
        this.bufferedJobs.sigCount += workReq.sets.length;
        if (this.bufferedJobs.sigCount > this.maxBufferedSigs) {
          clearTimeout(this.bufferedJobs.timeout);
          this.runBufferedJobs();
        }
      } else {
        this.jobs.push(job);
        setImmediate(this.runJob);
      }
    });
  }

  runBufferedJobs = () => {
    if (this.bufferedJobs) {
      this.jobs.push(...this.bufferedJobs.jobs);
      this.bufferedJobs = null;
      setImmediate(this.runJob);
    }
  };

  // Scheduled with setImmediate where index.ts uses setTimeout(runJob, 0): jobs queued in the
  // same macrotask still leave in one call, without Node's 1 ms floor on a zero timeout (a
  // whole millisecond on every gossip batch's critical path).
  // All queued jobs go to the device in one call; the library merges concurrent calls into
  // super-batches, so there is no idle-worker bookkeeping here (index.ts:290-381).
  runJob = async () => {
    if (this.closed || this.jobs.length === 0) return;
    const jobs = this.jobs.splice(0, this.jobs.length);
    const m = this.metrics ? this.metrics.blsThreadPool : null;
    let startedSigSets = 0;
    for (const job of jobs) {
      startedSigSets += job.workReq.sets.length;
      if (m) m.jobWaitTime.observe((Date.now() - job.addedTimeMs) / 1000);
    }
    if (m) {
      m.totalJobsGroupsStarted.inc(1);
      m.totalJobsStarted.inc(jobs.length);
      m.totalSigSetsStarted.inc(startedSigSets);
    }
    try {
      const codes = await addon.verify(
        this.ctx,
        jobs.map((j) => ({sets: j.workReq.sets, batchable: Boolean(j.workReq.opts.batchable)})),
        0
      );
      let successCount = 0;
      let errorCount = 0;
      jobs.forEach((job, i) => {
        const c = codes[i];
        if (c < 0) {
          errorCount += job.workReq.sets.length;
          job.reject(Error(addon.strerror(-c)));
        } else {
          successCount += job.workReq.sets.length;
          job.resolve(c === 1);
        }
      });
      const st = codes.stats || {batchRetries: 0, batchSigsSuccess: 0, deviceMs: 0};
      this.counters.successJobsSignatureSetsCount += successCount;
      this.counters.errorJobsSignatureSetsCount += errorCount;
      this.counters.batchRetries += st.batchRetries;
      if (m) {
        const jobTimeSec = st.deviceMs / 1000;
        m.timePerSigSet.observe(jobTimeSec / Math.max(1, startedSigSets));
        m.jobsWorkerTime.inc({workerId: 0}, jobTimeSec);
        m.successJobsSignatureSetsCount.inc(successCount);
        m.errorJobsSignatureSetsCount.inc(errorCount);
        m.batchRetries.inc(st.batchRetries);
        m.batchSigsSuccess.inc(st.batchSigsSuccess);
      }
    } catch (e) {
      for (const job of jobs) job.reject(e);
    }
  };

  // ---- SURVEY 8(f) entry points (synchronous; low volume beside verifySignatureSets) ----

  /** Light-client sync-aggregate check, isValidBlsAggregate (light-client/src/validation.ts:152-176):
   * PublicKey.aggregate(publicKeys) (throws on an empty list), then
   * Signature.fromBytes(signature, undefined, true).verify(aggPubkey, message) as one
   * non-batchable aggregate set: an undecodable or non-G2 signature throws with its BLST code,
   * an infinity aggregate verifies false. */
  async isValidBlsAggregate(publicKeys, message, signature) {
    if (publicKeys.length === 0) throw Error("EMPTY_AGGREGATE_ARRAY");
    return this.verifySignatureSets(
      [{type: SignatureSetType.aggregate, pubkeys: publicKeys, signingRoot: message, signature}],
      {batchable: false}
    );
  }

  /** bls.Signature.aggregate(sigs.map((s) => Signature.fromBytes(s, undefined, true))).toBytes()
   * (chain/opPools/attestationPool.ts:184-187): throws Error(BLST code) like the dependency. */
  aggregateSignatures(sigs) {
    return this.aggregateSignaturesMany([sigs])[0];
  }

  /** One aggregate per op-pool entry in a single device call; each element is the compressed
   * aggregate or an Error carrying the BLST code of its first failing signature. */
  aggregateSignaturesMany(aggregates) {
    const {status, sigs} = addon.aggregateSignatures(this.ctx, aggregates);
    return aggregates.map((_, a) => {
      if (status[a] < 0) throw Error(addon.strerror(-status[a]));
      return sigs.slice(96 * a, 96 * a + 96);
    });
  }

  /** Deposit-time key check, PublicKey.fromBytes(pk, affine, true) (processDeposit.ts:64):
   * per key null (valid) or the BLST code name. */
  validatePubkeys(keys48) {
    const flat = new Uint8Array(48 * keys48.length);
    keys48.forEach((k, i) => {
      if (k.length !== 48) throw Error("BLST_BAD_ENCODING");
      flat.set(k, 48 * i);
    });
    const {status} = addon.pubkeysValidate(this.ctx, flat);
    return Array.from(status, (c) => (c === 0 ? null : addon.strerror(-c)));
  }

  /** processDeposit.ts:62-70 signature check over {pubkey, signingRoot, signature} records. */
  verifyDeposits(deposits) {
    const n = deposits.length;
    const keys = new Uint8Array(48 * n);
    const roots = new Uint8Array(32 * n);
    const sigs = new Uint8Array(96 * n);
    deposits.forEach((d, i) => {
      keys.set(d.pubkey, 48 * i);
      roots.set(d.signingRoot, 32 * i);
      sigs.set(d.signature, 96 * i);
    });
    return Array.from(addon.depositsVerify(this.ctx, keys, roots, sigs), (v) => v === 1);
  }
}

function unwrap(code) {
  if (code < 0) throw Error(addon.strerror(-code));
  return code === 1;
}

module.exports = {BlsGpuVerifier, SignatureSetType, QueueError, chunkifyMaximizeChunkSize, getAggregatedPubkeysCount, toNativeSet, addon};
