"use strict";
/**
 * Chain options and CLI flags that select and tune BlsGpuVerifier.
 *
 * They sit beside the reference's BLS options: IChainOptions.blsVerifyAllMainThread /
 * blsVerifyAllMultiThread (packages/beacon-node/src/chain/options.ts:12-13, defaults :51-52)
 * and the hidden CLI flags chain.blsVerifyAllMainThread / chain.blsVerifyAllMultiThread
 * (packages/cli/src/options/beaconNodeOptions/chain.ts:6-8 IChainArgs, :25-27 parseArgs,
 * :58-74 options).  A beacon node spreads these three objects into its own:
 *   defaultChainOptions = {...defaultChainOptions, ...blsGpuChainOptionDefaults}
 *   parseArgs(args)     = {...parseArgs(args), ...parseBlsGpuArgs(args)}
 *   options             = {...options, ...blsGpuCliOptions}
 */

/** IChainOptions fields (index.d.ts BlsGpuChainOptions) and their defaults. */
const blsGpuChainOptionDefaults = Object.freeze({
  blsGpu: false,
  blsGpuDevices: undefined, // every visible HIP device
  blsGpuMaxBufferedSigs: undefined, // BlsGpuVerifier.js MAX_BUFFERED_SIGS
  blsGpuMaxBufferWaitMs: undefined, // BlsGpuVerifier.js MAX_BUFFER_WAIT_MS
});

/** yargs option definitions, keyed like the reference's "chain.*" flags. */
const blsGpuCliOptions = Object.freeze({
  "chain.blsGpu": {
    type: "boolean",
    description: "Verify BLS signature sets on MI355X GPUs (libblsgpu) instead of worker threads",
    defaultDescription: "false",
    group: "chain",
  },
  "chain.blsGpuDevices": {
    type: "array",
    description: "HIP device ordinals used by --chain.blsGpu (one context drives them all)",
    defaultDescription: "all visible devices",
    group: "chain",
  },
  "chain.blsGpuMaxBufferedSigs": {
    hidden: true,
    type: "number",
    description: "Buffered batchable signature sets that trigger a GPU call",
    group: "chain",
  },
  "chain.blsGpuMaxBufferWaitMs": {
    hidden: true,
    type: "number",
    description: "Longest wait of a buffered batchable job before it goes to the GPU",
    group: "chain",
  },
});

function toDeviceList(v) {
  if (v === undefined || v === null) return undefined;
  const list = (Array.isArray(v) ? v : String(v).split(",")).map((x) => Number(x));
  for (const d of list) {
    if (!Number.isInteger(d) || d < 0) throw Error(`Invalid --chain.blsGpuDevices entry: ${d}`);
  }
  return list;
}

/** CLI args ("chain.blsGpu", ...) -> the IChainOptions fields. */
function parseBlsGpuArgs(args) {
  return {
    blsGpu: args["chain.blsGpu"],
    blsGpuDevices: toDeviceList(args["chain.blsGpuDevices"]),
    blsGpuMaxBufferedSigs: args["chain.blsGpuMaxBufferedSigs"],
    blsGpuMaxBufferWaitMs: args["chain.blsGpuMaxBufferWaitMs"],
  };
}

module.exports = {blsGpuChainOptionDefaults, blsGpuCliOptions, parseBlsGpuArgs};
