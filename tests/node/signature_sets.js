"use strict";
// Drives lodestar_amd/node/signatureSets.js for tests/test_signature_sets.py.
//   node signature_sets.js sets   <case.json>   -> JSON list of produced sets (hex roots)
//   node signature_sets.js digest <versionHex> <gvrHex> -> fork digest hex
//   node signature_sets.js roots  <blocks.json> -> hash_tree_root of each SignedBeaconBlock's
//        message (snake_case consensus JSON, e.g. the reference's backfill blocks.json) and the
//        signing roots of its randao / proposer / attestation sets under mainnet domains
//   node signature_sets.js verify <case.json>   -> verifies the block's sets through
//        BlsGpuVerifier (GPU), prints {"valid": bool, "corrupt": bool}
const fs = require("fs");
const path = require("path");
const ss = require(path.join(__dirname, "..", "..", "lodestar_amd", "node", "signatureSets.js"));

const hex = (s) => Uint8Array.from(Buffer.from(s, "hex"));
const toHex = (b) => Buffer.from(b).toString("hex");

function header(h) {
  return {
    message: {
      slot: BigInt(h.slot),
      proposerIndex: h.proposerIndex,
      parentRoot: hex(h.parentRoot),
      stateRoot: hex(h.stateRoot),
      bodyRoot: hex(h.bodyRoot),
    },
    signature: hex(h.signature),
  };
}

function attData(d, big) {
  const n = big ? BigInt : Number;
  return {
    slot: n(d.slot),
    index: n(d.index),
    beaconBlockRoot: hex(d.beaconBlockRoot),
    source: {epoch: n(d.source.epoch), root: hex(d.source.root)},
    target: {epoch: n(d.target.epoch), root: hex(d.target.root)},
  };
}

function build(c) {
  const forks = c.forks.map((f) => ({name: f.name, epoch: f.epoch, version: hex(f.version)}));
  const config = ss.createForkConfig(forks, hex(c.genesisValidatorsRoot));
  const indexed = new Map();
  const attestations = c.block.attestations.map((a, i) => {
    const att = {aggregationBits: null, data: attData(a.data, false), signature: hex(a.signature), _id: i};
    indexed.set(att, {attestingIndices: a.attestingIndices, data: att.data, signature: att.signature});
    return att;
  });
  const state = {
    slot: c.stateSlot,
    config,
    epochCtx: {
      getIndexedAttestation: (att) => indexed.get(att),
      currentSyncCommitteeIndexed: {validatorIndices: c.syncCommittee},
    },
  };
  const b = c.block;
  const message = {
    slot: b.slot,
    proposerIndex: b.proposerIndex,
    parentRoot: hex(b.parentRoot),
    stateRoot: hex(b.stateRoot),
    bodyRoot: hex(b.bodyRoot),
    body: {
      randaoReveal: hex(b.randaoReveal),
      proposerSlashings: b.proposerSlashings.map((p) => ({signedHeader1: header(p[0]), signedHeader2: header(p[1])})),
      attesterSlashings: b.attesterSlashings.map((p) => ({
        attestation1: {attestingIndices: p[0].attestingIndices, data: attData(p[0].data, true), signature: hex(p[0].signature)},
        attestation2: {attestingIndices: p[1].attestingIndices, data: attData(p[1].data, true), signature: hex(p[1].signature)},
      })),
      attestations,
      voluntaryExits: b.voluntaryExits.map((x) => ({
        message: {epoch: x.epoch, validatorIndex: x.validatorIndex},
        signature: hex(x.signature),
      })),
      syncAggregate: b.syncAggregate
        ? {syncCommitteeBits: hex(b.syncAggregate.bits), syncCommitteeSignature: hex(b.syncAggregate.signature)}
        : undefined,
    },
  };
  return {state, signedBlock: {message, signature: hex(b.signature)}};
}

// ---- consensus JSON (snake_case, hex strings, decimal uint strings) -> reference JS shapes ----
const camel = (k) => k.replace(/_([a-z0-9])/g, (_, ch) => ch.toUpperCase());
function bitlistFromSsz(b) {
  // SSZ bitlist bytes end with a delimiter bit above the last data bit
  const last = b[b.length - 1];
  if (!last) throw Error("bitlist without delimiter");
  const top = 31 - Math.clz32(last);
  const bitLen = 8 * (b.length - 1) + top;
  const u = Uint8Array.from(b);
  u[u.length - 1] &= (1 << top) - 1;
  return {uint8Array: u, bitLen};
}
function fromJson(v, key) {
  if (Array.isArray(v)) return v.map((x) => fromJson(x, key));
  if (v && typeof v === "object") {
    const o = {};
    for (const k of Object.keys(v)) o[camel(k)] = fromJson(v[k], camel(k));
    return o;
  }
  if (typeof v === "string" && v.startsWith("0x")) {
    const b = hex(v.slice(2));
    return key === "aggregationBits" ? bitlistFromSsz(b) : b;
  }
  if (typeof v === "string" && /^[0-9]+$/.test(v)) return Number(v);
  return v;
}

const MAINNET_GVR = "4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95";
const MAINNET_FORKS = [
  {name: "phase0", epoch: 0, version: hex("00000000")},
  {name: "altair", epoch: 74240, version: hex("01000000")},
  {name: "bellatrix", epoch: 144896, version: hex("02000000")},
];

function roots(blocks) {
  const config = ss.createForkConfig(MAINNET_FORKS, hex(MAINNET_GVR));
  return blocks.map((j) => {
    const sb = fromJson(j);
    const state = {
      slot: sb.message.slot,
      config,
      epochCtx: {getIndexedAttestation: (a) => ({attestingIndices: [], data: a.data, signature: a.signature})},
    };
    const sets = ss.getBlockSignatureSets(state, sb);
    return {
      blockRoot: toHex(ss.ssz.BeaconBlock(sb.message)),
      bodyRoot: toHex(ss.ssz.BeaconBlockBody(sb.message.body)),
      sets: sets.map((s) => ({type: s.type, signingRoot: toHex(s.signingRoot)})),
    };
  });
}

function produce(c) {
  const {state, signedBlock} = build(c);
  return ss.getBlockSignatureSets(state, signedBlock, {skipProposerSignature: Boolean(c.skipProposerSignature)});
}

async function main() {
  const [mode, a, b] = process.argv.slice(2);
  if (mode === "digest") {
    process.stdout.write(toHex(ss.computeForkDigest(hex(a), hex(b))) + "\n");
    return;
  }
  const c = JSON.parse(fs.readFileSync(a, "utf8"));
  if (mode === "roots") {
    process.stdout.write(JSON.stringify(roots(c)) + "\n");
    return;
  }
  if (mode === "sets") {
    let out;
    try {
      out = produce(c).map((s) => ({
        type: s.type,
        indices: s.type === "single" ? [s.pubkey] : s.pubkeys,
        signingRoot: toHex(s.signingRoot),
        signature: toHex(s.signature),
      }));
    } catch (e) {
      out = {error: e.message};
    }
    process.stdout.write(JSON.stringify(out) + "\n");
    return;
  }
  if (mode === "verify") {
    const {BlsGpuVerifier, addon} = require(path.join(__dirname, "..", "..", "lodestar_amd", "node", "BlsGpuVerifier.js"));
    const v = new BlsGpuVerifier({devices: [0]});
    addon.keygen(v.ctx, hex(c.secretKeys), 0); // the case's validators at cache indices 0..n-1
    const sets = produce(c);
    // verifyBlocksSignatures.ts:34-48: one non-batchable call on the main thread path
    const valid = await v.verifySignatureSets(sets, {verifyOnMainThread: true});
    const bad = sets.slice();
    bad[1] = Object.assign({}, bad[1], {signingRoot: bad[2].signingRoot});
    const corrupt = await v.verifySignatureSets(bad, {verifyOnMainThread: true});
    await v.close();
    process.stdout.write(JSON.stringify({valid, corrupt, nsets: sets.length}) + "\n");
  }
}

main().catch((e) => {
  process.stderr.write(String(e && e.stack) + "\n");
  process.exit(1);
});
