/*
 * blsgpu.h — C-ABI of the MI355X batch BLS12-381 signature-set verifier
 * (libblsgpu.so).  Drop-in engine behind Lodestar's IBlsVerifier:
 *
 *   packages/beacon-node/src/chain/bls/interface.ts:20-46
 *     verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>
 *     close(): Promise<void>
 *
 * Each entry point below names the reference function it replaces.  The
 * reference holds no native code of its own: the arithmetic lives in the
 * un-vendored dependency @chainsafe/bls@7.1.1 -> @chainsafe/blst@0.2.4 ->
 * supranational blst (yarn.lock:458-473), which this library re-implements as
 * HIP kernels for gfx950.
 *
 * Conventions: plain C, no exceptions cross the boundary, every function
 * returns an int status (BGV_OK = 0, negative = call failed, see bgv_strerror).
 * Verdict codes per job are 1 (valid), 0 (invalid) or -code where code is one
 * of the BLST-numbered errors below.  One context per process; calls on one
 * context are serialised internally.
 */
#ifndef BLSGPU_H
#define BLSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes.  1..8 follow blst's BLST_ERROR enum (the message of the
 * rejected Promise contains the name, e.g. "BLST_INVALID_SIZE",
 * beacon-node/test/e2e/chain/bls/multithread.test.ts:86-103). */
enum {
  BGV_OK = 0,
  BGV_BLST_BAD_ENCODING = 1,
  BGV_BLST_POINT_NOT_ON_CURVE = 2,
  BGV_BLST_POINT_NOT_IN_GROUP = 3,
  BGV_BLST_AGGR_TYPE_MISMATCH = 4,
  BGV_BLST_VERIFY_FAIL = 5,
  BGV_BLST_PK_IS_INFINITY = 6,
  BGV_BLST_BAD_SCALAR = 7,
  BGV_BLST_INVALID_SIZE = 8,
  BGV_E_EMPTY_AGGREGATE = 20, /* PublicKey.aggregate([]) — "EMPTY_AGGREGATE_ARRAY" (chain/bls/utils.ts:11) */
  BGV_E_EMPTY_SET = 21,       /* "Empty signature set" (chain/bls/maybeBatch.ts:29-31) */
  BGV_E_BAD_INDEX = 22,       /* validator index not in the device pubkey cache */
  BGV_E_ARG = 23,             /* malformed call */
  BGV_E_DEVICE = 30,          /* HIP error: never reported as a verdict */
  BGV_E_NOMEM = 31,
  BGV_E_CLOSED = 32           /* QueueError QUEUE_ABORTED after close() (multithread/index.ts:176-186,239-241) */
};

/* Verification modes of bgv_verify. */
enum {
  /* BlsMultiThreadWorkerPool worker semantics (multithread/worker.ts:32-108):
   * batchable jobs are verified together, and when a device group that mixes
   * jobs fails, every job in it is re-verified alone; non-batchable jobs are
   * verified alone (no retry). */
  BGV_MODE_WORKER = 0,
  /* every job verified alone (verifySignatureSetsMaybeBatch per job,
   * maybeBatch.ts:16-39; also BlsSingleThreadVerifier, singleThread.ts:14-36) */
  BGV_MODE_PER_JOB = 1
};

/* Pubkey record formats for bgv_pubkeys_put. */
enum { BGV_PK_COMPRESSED = 48, BGV_PK_UNCOMPRESSED = 96 };

typedef struct bgv_ctx bgv_ctx;

/* One signature set: ISignatureSet (state-transition/src/util/signatureSets.ts:5-22).
 * single     -> n_pk = 1
 * aggregate  -> n_pk = pubkeys.length (0 rejects with BGV_E_EMPTY_AGGREGATE)
 * Pubkeys are trusted (already subgroup/infinity checked, interface.ts:33-36) and are
 * given either as validator indices into the device cache (pk_indices) or, for keys
 * not in the cache, as n_pk x 96-byte uncompressed records (pk_bytes, the
 * SerializedSet.publicKey format of multithread/types.ts:8-12). */
typedef struct {
  uint32_t n_pk;
  uint32_t sig_len;           /* length of sig as received; 96 is the only valid size */
  const uint32_t* pk_indices; /* n_pk indices, or NULL */
  const uint8_t* pk_bytes;    /* n_pk * 96 bytes when pk_indices is NULL */
  const uint8_t* msg;         /* 32-byte signing root */
  const uint8_t* sig;         /* compressed G2 signature, untrusted wire bytes */
} bgv_set;

/* One verifySignatureSets job (BlsWorkReq, multithread/types.ts:14-17): a
 * contiguous run of sets and its VerifySignatureOpts.batchable flag. */
typedef struct {
  uint32_t first_set;
  uint32_t n_sets;
  uint32_t batchable;
} bgv_job;

/* Counters mirroring BlsWorkResult (multithread/types.ts:24-36) plus device timing. */
typedef struct {
  uint64_t batch_retries;      /* mixed-job device groups that failed and were retried per job */
  uint64_t batch_sigs_success; /* sets verified valid in mixed-job groups */
  uint64_t device_groups;      /* device groups launched (each one final exponentiation) */
  uint64_t sets_verified;      /* slots launched, retries included */
  double device_ms;            /* HIP-event time of the kernels of this call */
  double wall_ms;              /* host wall time of the call */
} bgv_stats;

/* Create a context on the given HIP devices (NULL/0 = device 0).  Replaces the
 * pool constructor, multithread/index.ts:114-132. */
int bgv_init(const int* devices, int ndev, bgv_ctx** out);

/* Release all device memory.  After bgv_close() every call returns BGV_E_CLOSED. */
int bgv_close(bgv_ctx* ctx);
int bgv_destroy(bgv_ctx* ctx);

/* Upload validator pubkeys [first_index, first_index + n) into the device-resident
 * cache (replicated on every device).  fmt = BGV_PK_COMPRESSED (48-byte ZCash, as in
 * the beacon state) or BGV_PK_UNCOMPRESSED (96 bytes).  Keys are trusted: decoded
 * without a subgroup check, as Index2PubkeyCache does
 * (state-transition/src/cache/pubkeyCache.ts:56-77, epochContext.ts:702-705).
 * Appending (first_index == bgv_pubkeys_count) does not wait for running verifies: the keys
 * are decoded into staging memory and published once every device holds them.  A gap
 * (first_index > count) returns -BGV_E_ARG and writes nothing.  Undecodable records do not
 * stop the run: every index of it is committed, the undecodable ones are marked (a set that
 * names one rejects with BGV_E_BAD_INDEX) and -code of the first undecodable key is
 * returned; a later put over the same index replaces the mark. */
int bgv_pubkeys_put(bgv_ctx* ctx, uint32_t first_index, const uint8_t* keys, size_t n, int fmt);
size_t bgv_pubkeys_count(const bgv_ctx* ctx);

/* Verify njobs jobs over nsets sets; out_job_codes[j] receives 1, 0 or -error.
 * Replaces BlsMultiThreadWorkerPool.verifySignatureSets + the worker's
 * verifyManySignatureSets + verifySignatureSetsMaybeBatch
 * (multithread/index.ts:134-174, worker.ts:32-108, maybeBatch.ts:16-39).
 * stats may be NULL. */
int bgv_verify(bgv_ctx* ctx, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
               int32_t* out_job_codes, bgv_stats* stats);

/* Asynchronous form for the N-API addon (napi_async_work): the call runs on the
 * context's worker thread and `done(user, rc)` is invoked there when out_job_codes
 * and stats are filled.  The caller keeps every buffer alive until then. */
typedef void (*bgv_done_fn)(void* user, int rc);
int bgv_verify_async(bgv_ctx* ctx, const bgv_job* jobs, size_t njobs, const bgv_set* sets, size_t nsets, int mode,
                     int32_t* out_job_codes, bgv_stats* stats, bgv_done_fn done, void* user);

/* Parity hook for bls.PublicKey.aggregate + toBytes(uncompressed)
 * (chain/bls/utils.ts:5-16, multithread/index.ts:160): sum of cached pubkeys,
 * 96-byte uncompressed ZCash encoding (0x40 flag for infinity). */
int bgv_aggregate_pubkeys(bgv_ctx* ctx, const uint32_t* indices, size_t n, uint8_t out96[96]);

/* Parity hook for hash_to_G2 with DST BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_:
 * n messages (concatenated, lengths in lens) -> n x 192-byte uncompressed points
 * (x.c1 | x.c0 | y.c1 | y.c0). */
int bgv_hash_to_g2(bgv_ctx* ctx, const uint8_t* msgs, const uint32_t* lens, size_t n, uint8_t* out192);

/* Multi-GPU: one job's batch equation split over processes -------
 * The reference spreads a call's jobs over worker threads (multithread/index.ts:153-166);
 * here ONE job (e.g. a whole block range, or config 4 mode (ii)) can span GPUs.  Each rank
 * passes its shard of the job's sets to bgv_verify_partial, which returns the shard's
 * randomized Miller-loop product
 *     prod_i e(r_i pk_i, H(m_i)) * e(-G1, sum_i r_i sig_i)       (before the final exponentiation)
 * as 576 canonical big-endian bytes (the 12 Fp coefficients in tower order), and
 *     out_codes[0] = first signature error in set order (-BLST code) or 0,
 *     out_codes[1] = first pubkey condition: -BLST code, 1 for an infinity aggregate, or 0.
 * The partials are gathered (RCCL over xGMI, or gloo) and bgv_final_verify multiplies them
 * and runs ONE final exponentiation: *out_verdict = 1 iff the product is 1 in GT.
 * The job's outcome is then: the first nonzero signature code in rank order, else the
 * first pubkey code (1 = infinity aggregate: BLST_PK_IS_INFINITY for >= 2 sets, false for
 * one), else the verdict (lodestar_amd/shard.py). */
int bgv_verify_partial(bgv_ctx* ctx, const bgv_set* sets, size_t nsets, uint8_t out576[576], int32_t out_codes[2]);
/* One process over several devices: a context created on a device list spreads every
 * bgv_verify / bgv_verify_async call of at least min_sets sets over its devices -- a job of
 * at least min_sets sets as one run of sets per device whose Fp12 partials are combined with
 * one final exponentiation, the other jobs in contiguous runs pinned to one device each
 * (chain/bls/multithread/index.ts:153-166 splits big calls over workers the same way).
 * Codes are those of the unsplit call.  Default 4096 (BGV_SPLIT_MIN env); 0 disables. */
int bgv_set_split(bgv_ctx* ctx, uint32_t min_sets);
int bgv_final_verify(bgv_ctx* ctx, const uint8_t* partials, size_t n, int32_t* out_verdict);

/* Parity hook (tests only): the per-set intermediates of a verify call's kernels with the
 * path forced, so the latency path (which serves every call of up to 16,384 pairs: gossip,
 * block import) is checked byte for byte against the bulk path and the hash_to_G2 goldens.
 *   path 1 (BGV_PATH_BULK)     k_prep (task_hash/task_sig/task_pk), k_miller one pair per lane
 *   path 2 (BGV_PATH_LATENCY)  k_prep_a + k_prep_team, k_miller_team
 * The n sets (cached pubkeys only) form one job in groups of 64; set i gets the i-th nonzero
 * splitmix64 output from `seed` as its randomizer, so both paths see the same r_i.
 *   out_h192[i]    H(m_i), serialized like bgv_hash_to_g2
 *   out_f576[i]    its Miller-loop value f_i = e(r_i pk_i, H(m_i)) before the final
 *                  exponentiation (12 canonical big-endian Fp coefficients, tower order; 1 when
 *                  the set takes no part)
 *   out_status[2i], [2i+1]  the set's signature / pubkey status (0, 100 = infinity, or BLST code) */
#define BGV_PATH_BULK 1
#define BGV_PATH_LATENCY 2
int bgv_debug_prepare(bgv_ctx* ctx, const bgv_set* sets, size_t nsets, int path, uint64_t seed, uint8_t* out_h192,
                      uint8_t* out_f576, int32_t* out_status);

/* Parity hook for uniform groups (tests only; bgv_api.cpp call_submit / call_build_parts).
 * The n sets (2..64, cached pubkeys, one signing root, 96-B signatures) form ONE uniform
 * first-pass group of a bulk batch, randomizers as bgv_debug_prepare's; then ntests retry tests
 * over its slots, each a slot mask (bit k = set k), weighted (slot k with weight k + 1,
 * BGV_GROUP_WEIGHTED) when test_weighted[t] != 0.  Replaces the per-set pairs of a group whose
 * sets share a root, prod_i e(r_i pk_i, H) = e(sum_i r_i pk_i, H):
 *   out_first576       MillerLoop(sum_i r_i pk_i, H)                (k_gsum -> k_lines / k_facc)
 *   out_pk576[t]       MillerLoop(sum_{i in t} w_i r_i pk_i, H)     (k_gsum / k_gsum_w -> k_miller_team)
 *   out_sig576[t]      MillerLoop(-G1, sum_{i in t} w_i r_i sig_i)  (the test's signature pair)
 * 576-byte values as bgv_debug_prepare's f; w_i = 1, or i + 1 in a weighted test. */
int bgv_debug_uniform(bgv_ctx* ctx, const bgv_set* sets, size_t nsets, uint64_t seed, const uint64_t* test_masks,
                      const uint32_t* test_weighted, size_t ntests, uint8_t* out_first576, uint8_t* out_pk576,
                      uint8_t* out_sig576);

/* SURVEY 8(f) rows beside the verify path -------------------------------- */

/* Deposit-time pubkey validation: bls.PublicKey.fromBytes(pubkey, CoordType.affine,
 * validate=true) (state-transition/src/block/processDeposit.ts:64) for n 48-byte
 * compressed keys.  out_status[i] = 0 or -BLST code (BAD_ENCODING, POINT_NOT_ON_CURVE,
 * PK_IS_INFINITY, POINT_NOT_IN_GROUP).  out96 (may be NULL) receives the 96-byte
 * uncompressed record of every valid key (bgv_pubkeys_put / bgv_set.pk_bytes format). */
int bgv_pubkeys_validate(bgv_ctx* ctx, const uint8_t* keys48, size_t n, int32_t* out_status, uint8_t* out96);

/* Op-pool signature aggregation: bls.Signature.aggregate(sigs.map(s =>
 * Signature.fromBytes(s, undefined, true))) (chain/opPools/attestationPool.ts:184-187,
 * aggregatedAttestationPool.ts:319-321, syncCommitteeMessagePool.ts:126-129,
 * syncContributionAndProofPool.ts:181-185).  naggs aggregates over consecutive runs of
 * counts[a] signatures (96-byte records, lens[i] = the received length).  out96[a] is the
 * compressed aggregate, out_status[a] 0, -BLST code of the first signature that fails,
 * or -BGV_E_EMPTY_AGGREGATE for an empty run. */
int bgv_aggregate_signatures(bgv_ctx* ctx, const uint8_t* sigs96, const uint32_t* lens, const uint32_t* counts,
                             size_t naggs, uint8_t* out96, int32_t* out_status);

/* Deposit signature check (processDeposit.ts:62-70): key validated as above, then
 * Signature.fromBytes(sig, affine, true).verify(pk, signingRoot); any BLS error counts
 * as invalid.  out_valid[i] = 1 or 0. */
int bgv_deposits_verify(bgv_ctx* ctx, const uint8_t* keys48, const uint8_t* msgs32, const uint8_t* sigs96, size_t n,
                        int32_t* out_valid);

/* Bench/test utilities (not part of IBlsVerifier): derive public keys and sign on
 * the device.  sks are n x 32-byte big-endian secret keys (SecretKey.fromBytes).
 * bgv_keygen writes n x 48-byte compressed pubkeys to out48 (may be NULL) and, when
 * cache_first >= 0, stores them in the pubkey cache at [cache_first, cache_first + n).
 * bgv_sign writes n x 96-byte compressed signatures sk_i * H(msg_i) (msgs: n x 32 B). */
int bgv_keygen(bgv_ctx* ctx, const uint8_t* sks, size_t n, int64_t cache_first, uint8_t* out48);
int bgv_sign(bgv_ctx* ctx, const uint8_t* sks, const uint8_t* msgs, size_t n, uint8_t* out96);

/* Super-batch geometry: verify calls queued within coalesce_us of each other are merged
 * into one device launch of at most max_batch_slots sets (the GPU form of the pool's
 * MAX_BUFFERED_SIGS / MAX_BUFFER_WAIT_MS and prepareWork packaging,
 * multithread/index.ts:39-57,386-401).  While no super-batch is running the window is
 * idle_coalesce_us instead (at most coalesce_us), so a lone call launches at once.
 * max_batch_slots = 0 and a window of UINT32_MAX leave a value unchanged.  Defaults:
 * 131072 sets, 500 us, 50 us (env BGV_MAX_BATCH_SLOTS, BGV_COALESCE_US,
 * BGV_IDLE_COALESCE_US). */
int bgv_set_batching(bgv_ctx* ctx, uint32_t max_batch_slots, uint32_t coalesce_us, uint32_t idle_coalesce_us);

/* Deterministic batch randomizers for tests (seed != 0: splitmix64 stream;
 * seed == 0: getrandom(), the default). */
int bgv_set_rng_seed(bgv_ctx* ctx, uint64_t seed);

/* Per-kernel device time (HIP events between the kernels of each verify launch).
 * Reads the accumulated milliseconds per kernel (kernel_ms[n], names[n], launches)
 * and then, if enable >= 0, resets the counters and switches event recording on (1)
 * or off (0).  Returns the number of kernels in a verify launch. */
int bgv_profile(bgv_ctx* ctx, int enable, double* kernel_ms, const char** names, int n, uint64_t* launches);

/* Human-readable name of a status code ("BLST_INVALID_SIZE", ...). */
const char* bgv_strerror(int code);

int bgv_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* BLSGPU_H */
