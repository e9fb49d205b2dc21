"use strict";
/** Package entry (@lodestar/blsgpu): the verifier, its factory and its chain/CLI options.
 * BlsGpuVerifier (and with it the N-API addon) loads on first access. */
const {createBlsVerifier, createBlsGpuVerifier} = require("./createBlsVerifier.js");
const {blsGpuChainOptionDefaults, blsGpuCliOptions, parseBlsGpuArgs} = require("./chainOptions.js");

module.exports = {
  createBlsVerifier,
  createBlsGpuVerifier,
  blsGpuChainOptionDefaults,
  blsGpuCliOptions,
  parseBlsGpuArgs,
};
for (const name of ["BlsGpuVerifier", "SignatureSetType", "QueueError", "chunkifyMaximizeChunkSize"]) {
  Object.defineProperty(module.exports, name, {enumerable: true, get: () => require("./BlsGpuVerifier.js")[name]});
}
