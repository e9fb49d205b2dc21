"use strict";
/**
 * hash_tree_root for the consensus containers whose roots the signature-set producers sign
 * (consensus-specs ssz/simple-serialize.md "Merkleization"; the reference gets these from
 * @chainsafe/ssz through @lodestar/types' ssz.phase0 / ssz.altair namespaces).
 *
 * Values use the reference's JS shapes: uints as number or bigint, fixed byte vectors as
 * Uint8Array, bitlists / bitvectors as BitArray-like {uint8Array, bitLen} (bitLen of a
 * Bitvector is its length), lists as arrays, containers as camelCase objects.
 *
 * Pinned by the reference's backfill fixture of the first four mainnet blocks
 * (beacon-node/test/unit/sync/backfill/blocks.json, read in place by
 * tests/test_signature_sets.py): hash_tree_root(block[i]) == block[i+1].parent_root.
 */
const crypto = require("crypto");

// mainnet preset (packages/params/src/presets/mainnet.ts)
const P = {
  MAX_VALIDATORS_PER_COMMITTEE: 2048,
  MAX_PROPOSER_SLASHINGS: 16,
  MAX_ATTESTER_SLASHINGS: 2,
  MAX_ATTESTATIONS: 128,
  MAX_DEPOSITS: 16,
  MAX_VOLUNTARY_EXITS: 16,
  DEPOSIT_CONTRACT_TREE_DEPTH: 32,
  SYNC_COMMITTEE_SIZE: 512,
};

function hash(a, b) {
  return new Uint8Array(crypto.createHash("sha256").update(a).update(b).digest());
}

const ZERO = [new Uint8Array(32)]; // ZERO[d] = root of a depth-d all-zero tree
for (let d = 1; d < 64; d++) ZERO.push(hash(ZERO[d - 1], ZERO[d - 1]));

function depthOf(n) {
  let d = 0;
  while (2 ** d < n) d++;
  return d;
}

/** merkleize(chunks, limit): chunks padded with zero subtrees to next_pow2(limit || n) leaves */
function merkleize(chunks, limit) {
  const n = chunks.length;
  if (limit !== undefined && n > limit) throw Error("merkleize: " + n + " chunks over limit " + limit);
  const depth = depthOf(limit !== undefined ? Math.max(limit, 1) : Math.max(n, 1));
  let layer = chunks.slice();
  for (let d = 0; d < depth; d++) {
    const next = [];
    for (let i = 0; i < layer.length; i += 2) next.push(hash(layer[i], i + 1 < layer.length ? layer[i + 1] : ZERO[d]));
    layer = next;
    if (layer.length === 0) return ZERO[depth];
  }
  return layer.length ? layer[0] : ZERO[depth];
}

function mixInLength(root, length) {
  const l = Buffer.alloc(32);
  l.writeBigUInt64LE(BigInt(length), 0);
  return hash(root, l);
}

/** fixed bytes (Bytes4/32/48/96, Root, Version) packed into 32-byte chunks */
function packBytes(b) {
  const chunks = [];
  for (let i = 0; i < b.length; i += 32) {
    const c = new Uint8Array(32);
    c.set(b.subarray(i, Math.min(i + 32, b.length)));
    chunks.push(c);
  }
  return chunks.length ? chunks : [new Uint8Array(32)];
}

const bytesN = (len) => (b) => {
  if (b.length !== len) throw Error("expected " + len + " bytes, got " + b.length);
  return len <= 32 ? packBytes(b)[0] : merkleize(packBytes(b));
};

function uint64(v) {
  const c = Buffer.alloc(32);
  c.writeBigUInt64LE(BigInt(v), 0);
  return new Uint8Array(c);
}

function bitsBytes(bits, bitLen) {
  const out = new Uint8Array(Math.ceil(bitLen / 8));
  out.set(bits.subarray(0, out.length));
  if (bitLen % 8) out[out.length - 1] &= (1 << bitLen % 8) - 1;
  return out;
}

const bitlist = (limit) => (ba) =>
  mixInLength(merkleize(packBytes(bitsBytes(ba.uint8Array, ba.bitLen)).slice(0, Math.ceil(ba.bitLen / 256) || 0),
    Math.ceil(limit / 256)), ba.bitLen);

const bitvector = (len) => (ba) => merkleize(packBytes(bitsBytes(ba.uint8Array || ba, len)), Math.ceil(len / 256));

const list = (elem, limit) => (xs) => mixInLength(merkleize(xs.map(elem), limit), xs.length);

/** List[uint64, limit]: 4 values per chunk */
const uint64List = (limit) => (xs) => {
  const b = Buffer.alloc(8 * xs.length);
  xs.forEach((v, i) => b.writeBigUInt64LE(BigInt(v), 8 * i));
  const chunks = xs.length ? packBytes(new Uint8Array(b)) : [];
  return mixInLength(merkleize(chunks, Math.ceil((8 * limit) / 32)), xs.length);
};

const vector = (elem) => (xs) => merkleize(xs.map(elem));

/** container: fields in declaration order, [name, type] */
const container = (fields) => (v) => merkleize(fields.map(([k, t]) => t(v[k])));

const Root = bytesN(32);
const Bytes4 = bytesN(4);
const Bytes48 = bytesN(48);
const Bytes96 = bytesN(96);

const Checkpoint = container([["epoch", uint64], ["root", Root]]);
const AttestationData = container([
  ["slot", uint64],
  ["index", uint64],
  ["beaconBlockRoot", Root],
  ["source", Checkpoint],
  ["target", Checkpoint],
]);
const BeaconBlockHeader = container([
  ["slot", uint64],
  ["proposerIndex", uint64],
  ["parentRoot", Root],
  ["stateRoot", Root],
  ["bodyRoot", Root],
]);
const SignedBeaconBlockHeader = container([["message", BeaconBlockHeader], ["signature", Bytes96]]);
const ProposerSlashing = container([["signedHeader1", SignedBeaconBlockHeader], ["signedHeader2", SignedBeaconBlockHeader]]);
const IndexedAttestation = container([
  ["attestingIndices", uint64List(P.MAX_VALIDATORS_PER_COMMITTEE)],
  ["data", AttestationData],
  ["signature", Bytes96],
]);
const AttesterSlashing = container([["attestation1", IndexedAttestation], ["attestation2", IndexedAttestation]]);
const Attestation = container([
  ["aggregationBits", bitlist(P.MAX_VALIDATORS_PER_COMMITTEE)],
  ["data", AttestationData],
  ["signature", Bytes96],
]);
const DepositData = container([
  ["pubkey", Bytes48],
  ["withdrawalCredentials", Root],
  ["amount", uint64],
  ["signature", Bytes96],
]);
const DepositMessage = container([["pubkey", Bytes48], ["withdrawalCredentials", Root], ["amount", uint64]]);
const Deposit = container([["proof", vector(Root)], ["data", DepositData]]);
const VoluntaryExit = container([["epoch", uint64], ["validatorIndex", uint64]]);
const SignedVoluntaryExit = container([["message", VoluntaryExit], ["signature", Bytes96]]);
const Eth1Data = container([["depositRoot", Root], ["depositCount", uint64], ["blockHash", Root]]);
const SyncAggregate = container([
  ["syncCommitteeBits", bitvector(P.SYNC_COMMITTEE_SIZE)],
  ["syncCommitteeSignature", Bytes96],
]);

const phase0BodyFields = [
  ["randaoReveal", Bytes96],
  ["eth1Data", Eth1Data],
  ["graffiti", Root],
  ["proposerSlashings", list(ProposerSlashing, P.MAX_PROPOSER_SLASHINGS)],
  ["attesterSlashings", list(AttesterSlashing, P.MAX_ATTESTER_SLASHINGS)],
  ["attestations", list(Attestation, P.MAX_ATTESTATIONS)],
  ["deposits", list(Deposit, P.MAX_DEPOSITS)],
  ["voluntaryExits", list(SignedVoluntaryExit, P.MAX_VOLUNTARY_EXITS)],
];
const Phase0BeaconBlockBody = container(phase0BodyFields);
const AltairBeaconBlockBody = container(phase0BodyFields.concat([["syncAggregate", SyncAggregate]]));
/** phase0 or altair body, told apart by syncAggregate (later forks: pass the node's ssz types) */
const BeaconBlockBody = (b) => (b.syncAggregate ? AltairBeaconBlockBody(b) : Phase0BeaconBlockBody(b));

function BeaconBlock(b) {
  return BeaconBlockHeader({
    slot: b.slot,
    proposerIndex: b.proposerIndex,
    parentRoot: b.parentRoot,
    stateRoot: b.stateRoot,
    bodyRoot: b.bodyRoot || BeaconBlockBody(b.body),
  });
}

const ForkData = container([["currentVersion", Bytes4], ["genesisValidatorsRoot", Root]]);
const SigningData = container([["objectRoot", Root], ["domain", Root]]);

module.exports = {
  preset: P,
  ZERO_HASHES: ZERO,
  merkleize,
  mixInLength,
  uint64,
  Root,
  Bytes4,
  Bytes48,
  Bytes96,
  Epoch: uint64,
  Checkpoint,
  AttestationData,
  AttestationDataBigint: AttestationData,
  BeaconBlockHeader,
  BeaconBlockHeaderBigint: BeaconBlockHeader,
  ProposerSlashing,
  IndexedAttestation,
  AttesterSlashing,
  Attestation,
  DepositData,
  DepositMessage,
  Deposit,
  VoluntaryExit,
  SignedVoluntaryExit,
  Eth1Data,
  SyncAggregate,
  Phase0BeaconBlockBody,
  AltairBeaconBlockBody,
  BeaconBlockBody,
  BeaconBlock,
  ForkData,
  SigningData,
};
