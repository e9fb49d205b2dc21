"use strict";
/**
 * Signature-set producers that emit validator INDICES (SURVEY §8(f)3).
 *
 * Restates packages/state-transition/src/signatureSets/ with one change: where the reference
 * resolves every index through epochCtx.index2pubkey[i] to a PublicKey object (randao.ts:30,
 * proposer.ts:28, proposerSlashings.ts:14, attesterSlashings.ts:36, indexedAttestation.ts:17,
 * voluntaryExits.ts:32, block/processSyncCommittee.ts:95), the sets here carry the index itself.
 * BlsGpuVerifier (toNativeSet) passes indices straight to the device-resident pubkey cache, so
 * a block's 16k attesting keys are never materialised as JS objects or aggregated on the main
 * thread.  Set order, domains, signing roots and the empty-sync-aggregate rule are the
 * reference's:
 *
 *   getBlockSignatureSets               signatureSets/index.ts:23-56
 *   getRandaoRevealSignatureSet         signatureSets/randao.ts:19-34
 *   getProposerSignatureSet             signatureSets/proposer.ts:15-32
 *   getProposerSlashing(s)SignatureSets signatureSets/proposerSlashings.ts:9-43
 *   getAttesterSlashing(s)SignatureSets signatureSets/attesterSlashings.ts:7-40
 *   getAttestationWithIndicesSignatureSet / getIndexedAttestationSignatureSet /
 *   getAttestationsSignatureSets        signatureSets/indexedAttestation.ts:6-37
 *   getVoluntaryExit(s)SignatureSet(s)  signatureSets/voluntaryExits.ts:22-45
 *   getSyncCommitteeSignatureSet        block/processSyncCommittee.ts:46-99
 *
 * `state` is duck-typed like CachedBeaconStateAllForks for the fields these functions read:
 *   state.slot
 *   state.config.getDomain(stateSlot, domainType, messageSlot?)   (createForkConfig below, or
 *       the node's IBeaconConfig) and state.config.ALTAIR_FORK_EPOCH
 *   state.epochCtx.getIndexedAttestation(attestation) -> {attestingIndices, data, signature}
 *   state.epochCtx.currentSyncCommitteeIndexed.validatorIndices
 * and `types` optionally maps SSZ type names (Epoch, Root, AttestationData(Bigint),
 * BeaconBlockHeader(Bigint), VoluntaryExit, BeaconBlock) to the node's fork-specific ssz types
 * (objects with hashTreeRoot) or functions; the defaults are ssz.js (phase0 / altair).
 */
const SLOTS_PER_EPOCH = 32;
const DOMAIN_BEACON_PROPOSER = Uint8Array.of(0, 0, 0, 0);
const DOMAIN_BEACON_ATTESTER = Uint8Array.of(1, 0, 0, 0);
const DOMAIN_RANDAO = Uint8Array.of(2, 0, 0, 0);
const DOMAIN_VOLUNTARY_EXIT = Uint8Array.of(4, 0, 0, 0);
const DOMAIN_SYNC_COMMITTEE = Uint8Array.of(7, 0, 0, 0);
const G2_POINT_AT_INFINITY = (() => {
  const b = new Uint8Array(96);
  b[0] = 0xc0;
  return b;
})();
const SignatureSetType = {single: "single", aggregate: "aggregate"};

const ssz = require("./ssz.js");

// hash_tree_root by SSZ type name (ssz.js; the node passes its own @lodestar/types ssz to
// cover later forks' block bodies)
const defaultTypes = ssz;

function bytesRoot(b, len) {
  if (b.length !== len) throw Error("expected " + len + " bytes, got " + b.length);
  return Uint8Array.from(b);
}

/** compute_signing_root: hash_tree_root(SigningData{object_root, domain}) (util/signingRoot.ts) */
function computeSigningRoot(objectRoot, domain) {
  return ssz.SigningData({objectRoot: bytesRoot(objectRoot, 32), domain: bytesRoot(domain, 32)});
}

/** compute_fork_data_root: hash_tree_root(ForkData{current_version, genesis_validators_root}) */
function computeForkDataRoot(version, genesisValidatorsRoot) {
  return ssz.ForkData({currentVersion: version, genesisValidatorsRoot});
}

function computeForkDigest(version, genesisValidatorsRoot) {
  return computeForkDataRoot(version, genesisValidatorsRoot).slice(0, 4);
}

/** compute_domain (config/src/genesisConfig/index.ts computeDomain) */
function computeDomain(domainType, forkVersion, genesisValidatorsRoot) {
  const out = new Uint8Array(32);
  out.set(domainType, 0);
  out.set(computeForkDataRoot(forkVersion, genesisValidatorsRoot).slice(0, 28), 4);
  return out;
}

const computeEpochAtSlot = (slot) => Math.floor(slot / SLOTS_PER_EPOCH);
const computeStartSlotAtEpoch = (epoch) => epoch * SLOTS_PER_EPOCH;

/**
 * The getDomain of createICachedGenesis (config/src/genesisConfig/index.ts:27-54) over a fork
 * schedule [{name, epoch, version}] sorted by epoch: the message epoch selects the fork at
 * stateSlot or the one before it.
 */
function createForkConfig(forks, genesisValidatorsRoot) {
  const sorted = forks.slice().sort((a, b) => a.epoch - b.epoch);
  const cache = new Map();
  const altair = sorted.find((f) => f.name === "altair");
  return {
    ALTAIR_FORK_EPOCH: altair ? altair.epoch : Infinity,
    getForkInfo(slot) {
      const epoch = computeEpochAtSlot(slot);
      let i = 0;
      while (i + 1 < sorted.length && sorted[i + 1].epoch <= epoch) i++;
      return {current: sorted[i], prev: sorted[Math.max(0, i - 1)]};
    },
    getDomain(stateSlot, domainType, messageSlot) {
      const epoch = computeEpochAtSlot(messageSlot === undefined || messageSlot === null ? stateSlot : messageSlot);
      const info = this.getForkInfo(stateSlot);
      const fork = epoch < info.current.epoch ? info.prev : info.current;
      const key = fork.name + ":" + Buffer.from(domainType).toString("hex");
      let d = cache.get(key);
      if (!d) {
        d = computeDomain(domainType, fork.version, genesisValidatorsRoot);
        cache.set(key, d);
      }
      return d;
    },
  };
}

// ---- producers ------------------------------------------------------------------------------

function rootOf(types, name, value) {
  const t = (types && types[name]) || defaultTypes[name];
  // a @chainsafe/ssz type object (node) or a hash_tree_root function (ssz.js)
  return typeof t === "function" ? t(value) : t.hashTreeRoot(value);
}

/** randao.ts:19-34 */
function getRandaoRevealSignatureSet(state, block, types) {
  const epoch = computeEpochAtSlot(block.slot);
  const domain = state.config.getDomain(state.slot, DOMAIN_RANDAO, block.slot);
  return {
    type: SignatureSetType.single,
    pubkey: block.proposerIndex,
    signingRoot: computeSigningRoot(rootOf(types, "Epoch", epoch), domain),
    signature: block.body.randaoReveal,
  };
}

/** proposer.ts:15-32 (blinded blocks hash with the blinded type: pass types.BeaconBlock) */
function getProposerSignatureSet(state, signedBlock, types) {
  const domain = state.config.getDomain(state.slot, DOMAIN_BEACON_PROPOSER, signedBlock.message.slot);
  return {
    type: SignatureSetType.single,
    pubkey: signedBlock.message.proposerIndex,
    signingRoot: computeSigningRoot(rootOf(types, "BeaconBlock", signedBlock.message), domain),
    signature: signedBlock.signature,
  };
}

/** proposerSlashings.ts:9-34: both headers signed by the same proposer */
function getProposerSlashingSignatureSets(state, proposerSlashing, types) {
  const index = proposerSlashing.signedHeader1.message.proposerIndex;
  return [proposerSlashing.signedHeader1, proposerSlashing.signedHeader2].map((signedHeader) => {
    const domain = state.config.getDomain(state.slot, DOMAIN_BEACON_PROPOSER, Number(signedHeader.message.slot));
    return {
      type: SignatureSetType.single,
      pubkey: index,
      signingRoot: computeSigningRoot(rootOf(types, "BeaconBlockHeaderBigint", signedHeader.message), domain),
      signature: signedHeader.signature,
    };
  });
}

function getProposerSlashingsSignatureSets(state, signedBlock, types) {
  const out = [];
  for (const ps of signedBlock.message.body.proposerSlashings) out.push(...getProposerSlashingSignatureSets(state, ps, types));
  return out;
}

/** attesterSlashings.ts:26-40 */
function getIndexedAttestationBigintSignatureSet(state, indexedAttestation, types) {
  const slot = computeStartSlotAtEpoch(Number(indexedAttestation.data.target.epoch));
  const domain = state.config.getDomain(state.slot, DOMAIN_BEACON_ATTESTER, slot);
  return {
    type: SignatureSetType.aggregate,
    pubkeys: Array.from(indexedAttestation.attestingIndices, Number),
    signingRoot: computeSigningRoot(rootOf(types, "AttestationDataBigint", indexedAttestation.data), domain),
    signature: indexedAttestation.signature,
  };
}

/** attesterSlashings.ts:17-24 */
function getAttesterSlashingSignatureSets(state, attesterSlashing, types) {
  return [attesterSlashing.attestation1, attesterSlashing.attestation2].map((a) =>
    getIndexedAttestationBigintSignatureSet(state, a, types)
  );
}

function getAttesterSlashingsSignatureSets(state, signedBlock, types) {
  const out = [];
  for (const as of signedBlock.message.body.attesterSlashings) out.push(...getAttesterSlashingSignatureSets(state, as, types));
  return out;
}

/** indexedAttestation.ts:6-21 */
function getAttestationWithIndicesSignatureSet(state, attestation, indices, types) {
  const slot = computeStartSlotAtEpoch(attestation.data.target.epoch);
  const domain = state.config.getDomain(state.slot, DOMAIN_BEACON_ATTESTER, slot);
  return {
    type: SignatureSetType.aggregate,
    pubkeys: Array.from(indices),
    signingRoot: computeSigningRoot(rootOf(types, "AttestationData", attestation.data), domain),
    signature: attestation.signature,
  };
}

/** indexedAttestation.ts:23-28 */
function getIndexedAttestationSignatureSet(state, indexedAttestation, types) {
  return getAttestationWithIndicesSignatureSet(state, indexedAttestation, indexedAttestation.attestingIndices, types);
}

/** indexedAttestation.ts:30-37 */
function getAttestationsSignatureSets(state, signedBlock, types) {
  return signedBlock.message.body.attestations.map((attestation) =>
    getIndexedAttestationSignatureSet(state, state.epochCtx.getIndexedAttestation(attestation), types)
  );
}

/** voluntaryExits.ts:22-36 */
function getVoluntaryExitSignatureSet(state, signedVoluntaryExit, types) {
  const slot = computeStartSlotAtEpoch(signedVoluntaryExit.message.epoch);
  const domain = state.config.getDomain(state.slot, DOMAIN_VOLUNTARY_EXIT, slot);
  return {
    type: SignatureSetType.single,
    pubkey: signedVoluntaryExit.message.validatorIndex,
    signingRoot: computeSigningRoot(rootOf(types, "VoluntaryExit", signedVoluntaryExit.message), domain),
    signature: signedVoluntaryExit.signature,
  };
}

function getVoluntaryExitsSignatureSets(state, signedBlock, types) {
  return signedBlock.message.body.voluntaryExits.map((x) => getVoluntaryExitSignatureSet(state, x, types));
}

/** SSZ Bitvector (LSB-first within each byte) or a BitArray with intersectValues */
function intersectBits(bits, values) {
  if (bits && typeof bits.intersectValues === "function") return bits.intersectValues(values);
  const bytes = bits.uint8Array || bits;
  const out = [];
  for (let i = 0; i < values.length; i++) if ((bytes[i >> 3] >> (i & 7)) & 1) out.push(values[i]);
  return out;
}

function bytesEqual(a, b) {
  if (a.length !== b.length) return false;
  for (let i = 0; i < a.length; i++) if (a[i] !== b[i]) return false;
  return true;
}

/** block/processSyncCommittee.ts:46-99: null when nobody participated (and the signature is
 * the point at infinity), else one aggregate set over the participants' indices */
function getSyncCommitteeSignatureSet(state, block, participantIndices, types) {
  const {syncAggregate} = block.body;
  const signature = syncAggregate.syncCommitteeSignature;
  const previousSlot = Math.max(block.slot, 1) - 1;
  const rootSigned = block.parentRoot;
  if (!participantIndices) {
    const committeeIndices = state.epochCtx.currentSyncCommitteeIndexed.validatorIndices;
    participantIndices = intersectBits(syncAggregate.syncCommitteeBits, committeeIndices);
  }
  if (participantIndices.length === 0) {
    if (bytesEqual(signature, G2_POINT_AT_INFINITY)) return null;
    throw Error("Empty sync committee signature is not infinity");
  }
  const domain = state.config.getDomain(state.slot, DOMAIN_SYNC_COMMITTEE, previousSlot);
  return {
    type: SignatureSetType.aggregate,
    pubkeys: Array.from(participantIndices),
    signingRoot: computeSigningRoot(rootOf(types, "Root", rootSigned), domain),
    signature,
  };
}

/** index.ts:23-56: randao, proposer slashings, attester slashings, attestations, exits,
 * [proposer], [sync aggregate] — deposits excluded (they may carry invalid signatures) */
function getBlockSignatureSets(state, signedBlock, opts, types) {
  const sets = [
    getRandaoRevealSignatureSet(state, signedBlock.message, types),
    ...getProposerSlashingsSignatureSets(state, signedBlock, types),
    ...getAttesterSlashingsSignatureSets(state, signedBlock, types),
    ...getAttestationsSignatureSets(state, signedBlock, types),
    ...getVoluntaryExitsSignatureSets(state, signedBlock, types),
  ];
  if (!(opts && opts.skipProposerSignature)) sets.push(getProposerSignatureSet(state, signedBlock, types));
  if (computeEpochAtSlot(signedBlock.message.slot) >= state.config.ALTAIR_FORK_EPOCH) {
    const sync = getSyncCommitteeSignatureSet(state, signedBlock.message, undefined, types);
    if (sync) sets.push(sync);
  }
  return sets;
}

module.exports = {
  SignatureSetType,
  SLOTS_PER_EPOCH,
  DOMAIN_BEACON_PROPOSER,
  DOMAIN_BEACON_ATTESTER,
  DOMAIN_RANDAO,
  DOMAIN_VOLUNTARY_EXIT,
  DOMAIN_SYNC_COMMITTEE,
  G2_POINT_AT_INFINITY,
  ssz,
  computeSigningRoot,
  computeForkDataRoot,
  computeForkDigest,
  computeDomain,
  computeEpochAtSlot,
  computeStartSlotAtEpoch,
  createForkConfig,
  getBlockSignatureSets,
  getRandaoRevealSignatureSet,
  getProposerSignatureSet,
  getProposerSlashingSignatureSets,
  getProposerSlashingsSignatureSets,
  getAttesterSlashingSignatureSets,
  getAttesterSlashingsSignatureSets,
  getIndexedAttestationBigintSignatureSet,
  getAttestationWithIndicesSignatureSet,
  getIndexedAttestationSignatureSet,
  getAttestationsSignatureSets,
  getVoluntaryExitSignatureSet,
  getVoluntaryExitsSignatureSets,
  getSyncCommitteeSignatureSet,
};
