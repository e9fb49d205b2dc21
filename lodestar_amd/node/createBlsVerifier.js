"use strict";
/**
 * Verifier selection for BeaconChain: the reference picks BlsSingleThreadVerifier when
 * opts.blsVerifyAllMainThread is set, else BlsMultiThreadWorkerPool
 * (packages/beacon-node/src/chain/chain.ts:189-192).  createBlsVerifier adds the GPU branch:
 * with opts.blsGpu (and not blsVerifyAllMainThread) it builds BlsGpuVerifier and installs its
 * pubkey-added hook before the chain's first syncPubkeys, so every validator key reaches the
 * device cache (INTEGRATION.md §2).
 *
 * The two CPU implementations live in the beacon node; the caller passes their constructors
 * ({BlsSingleThreadVerifier, BlsMultiThreadWorkerPool}), so this module carries none of the
 * reference's code and loads the GPU addon only when the GPU branch is taken.
 */

/**
 * @param {object} opts IChainOptions (blsVerifyAllMainThread, blsVerifyAllMultiThread, blsGpu*)
 * @param {object} modules {metrics, logger} as the reference passes them
 * @param {object} impls {BlsSingleThreadVerifier, BlsMultiThreadWorkerPool, setPubkeyAddedHook}
 */
function createBlsVerifier(opts, modules, impls = {}) {
  if (opts.blsVerifyAllMainThread) {
    if (!impls.BlsSingleThreadVerifier) throw Error("createBlsVerifier: BlsSingleThreadVerifier not provided");
    return new impls.BlsSingleThreadVerifier({metrics: modules.metrics});
  }
  if (opts.blsGpu) return createBlsGpuVerifier(opts, modules, impls.setPubkeyAddedHook);
  if (!impls.BlsMultiThreadWorkerPool) throw Error("createBlsVerifier: BlsMultiThreadWorkerPool not provided");
  return new impls.BlsMultiThreadWorkerPool(opts, modules);
}

/** BlsGpuVerifier from the chain options; installs the pubkey hook when one is given. */
function createBlsGpuVerifier(opts, modules = {}, setPubkeyAddedHook) {
  const {BlsGpuVerifier} = require("./BlsGpuVerifier.js");
  const verifier = new BlsGpuVerifier(
    {
      devices: opts.blsGpuDevices,
      maxBufferedSigs: opts.blsGpuMaxBufferedSigs,
      maxBufferWaitMs: opts.blsGpuMaxBufferWaitMs,
      blsVerifyAllMultiThread: opts.blsVerifyAllMultiThread,
    },
    {metrics: modules.metrics || null}
  );
  if (setPubkeyAddedHook) setPubkeyAddedHook(verifier.pubkeyAddedHook());
  return verifier;
}

module.exports = {createBlsVerifier, createBlsGpuVerifier};
