"""Index-emitting signature-set producers (lodestar_amd/node/signatureSets.js)
driven through Node.

* SSZ roots pinned by the reference's own fixture, read in place (CPU only; skipped where
  /root/reference is absent): the first four mainnet blocks of
  beacon-node/test/unit/sync/backfill/blocks.json, hash_tree_root(block[i]) ==
  block[i+1].parent_root.
* Fork digests of mainnet (ForkData roots) against the published values: phase0 b5303f2a,
  altair afcaaba0, bellatrix 4a26c58b (the last also in network/gossip/scoringParameters.ts:178).
* The reference's unit test (state-transition/test/unit/signatureSets/signatureSets.test.ts:16-81)
  restated: one proposer slashing, one attester slashing, one attestation and one exit give
  7 sets; plus the altair sync-aggregate rules (processSyncCommittee.ts:75-99).
* Every produced set's signing root equals an independent Python restatement of
  compute_signing_root / compute_domain (below) and carries validator indices, in the
  reference's order; on the GPU the sets, signed with interop keys, verify through
  BlsGpuVerifier (one non-batchable call, verifyBlocksSignatures.ts:34-48) and a swapped
  root fails.
"""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tests", "node", "signature_sets.js")
MAINNET_BLOCKS = "/root/reference/packages/beacon-node/test/unit/sync/backfill/blocks.json"
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
MAINNET_GVR = "4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95"

pytestmark = pytest.mark.skipif(shutil.which("node") is None, reason="node not in image")


def node(*args, timeout=120):
    p = subprocess.run(["node", SCRIPT] + list(args), cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr
    return p.stdout.strip()


# ---- independent Python restatement of the signing-root arithmetic ---------------------------
def h(a, b):
    return hashlib.sha256(a + b).digest()


def merkle(chunks):
    n = 1
    while n < len(chunks):
        n *= 2
    layer = list(chunks) + [bytes(32)] * (n - len(chunks))
    while len(layer) > 1:
        layer = [h(layer[i], layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def u64(v):
    return int(v).to_bytes(8, "little") + bytes(24)


def domain(dtype, version, gvr):
    return bytes([dtype, 0, 0, 0]) + merkle([version + bytes(28), gvr])[:28]


def signing_root(obj_root, dom):
    return merkle([obj_root, dom])


def att_data_root(d):
    ck = lambda c: merkle([u64(c["epoch"]), bytes.fromhex(c["root"])])  # noqa: E731
    return merkle([u64(d["slot"]), u64(d["index"]), bytes.fromhex(d["beaconBlockRoot"]), ck(d["source"]),
                   ck(d["target"])])


def header_root(x):
    return merkle([u64(x["slot"]), u64(x["proposerIndex"]), bytes.fromhex(x["parentRoot"]),
                   bytes.fromhex(x["stateRoot"]), bytes.fromhex(x["bodyRoot"])])


# ---- a block case -------------------------------------------------------------------------------
def _root(tag):
    return hashlib.sha256(tag.encode()).hexdigest()


def _att(slot, index, target_epoch, indices, sig="00" * 96):
    return {"data": {"slot": slot, "index": index, "beaconBlockRoot": _root("bbr%d" % slot),
                     "source": {"epoch": max(0, target_epoch - 1), "root": _root("src")},
                     "target": {"epoch": target_epoch, "root": _root("tgt%d" % target_epoch)}},
            "attestingIndices": indices, "signature": sig}


def _hdr(slot, proposer, tag):
    return {"slot": slot, "proposerIndex": proposer, "parentRoot": _root("p" + tag), "stateRoot": _root("s" + tag),
            "bodyRoot": _root("b" + tag), "signature": "00" * 96}


def make_case(altair_epoch=1, sync_bits=None, sync_sig=None, slot=40, skip_proposer=False):
    committee = [3, 5, 7, 9, 11, 13, 15, 2]
    bits = sync_bits if sync_bits is not None else [1, 0, 1, 1, 0, 0, 1, 0]
    bitbytes = bytearray(64)  # Bitvector[512]
    for i, b in enumerate(bits):
        if b:
            bitbytes[i >> 3] |= 1 << (i & 7)
    return {
        "forks": [{"name": "phase0", "epoch": 0, "version": "00000000"},
                  {"name": "altair", "epoch": altair_epoch, "version": "01000000"}],
        "genesisValidatorsRoot": MAINNET_GVR,
        "stateSlot": slot,
        "syncCommittee": committee,
        "skipProposerSignature": skip_proposer,
        "block": {
            "slot": slot, "proposerIndex": 4, "parentRoot": _root("parent"), "stateRoot": _root("state"),
            "bodyRoot": _root("body"), "randaoReveal": "00" * 96, "signature": "00" * 96,
            "proposerSlashings": [[_hdr(33, 6, "1"), _hdr(33, 6, "2")]],
            "attesterSlashings": [[_att(1, 0, 0, [1, 8, 12]), _att(1, 0, 0, [8, 12, 14])]],
            "attestations": [_att(39, 1, 1, [0, 10, 14]), _att(31, 0, 0, [1, 2])],
            "voluntaryExits": [{"epoch": 1, "validatorIndex": 9, "signature": "00" * 96}],
            "syncAggregate": {"bits": bytes(bitbytes).hex(),
                              "signature": sync_sig if sync_sig is not None else "00" * 96},
        },
    }


def expected_sets(c):
    """(type, indices, signing root) in getBlockSignatureSets order, from the Python restatement."""
    gvr = bytes.fromhex(c["genesisValidatorsRoot"])
    forks = sorted(c["forks"], key=lambda f: f["epoch"])

    def dom(dtype, msg_slot):
        st_epoch, epoch = c["stateSlot"] // 32, msg_slot // 32
        i = max(k for k, f in enumerate(forks) if f["epoch"] <= st_epoch)
        f = forks[i] if epoch >= forks[i]["epoch"] else forks[max(0, i - 1)]
        return domain(dtype, bytes.fromhex(f["version"]), gvr)

    b = c["block"]
    out = [("single", [b["proposerIndex"]], signing_root(u64(b["slot"] // 32), dom(2, b["slot"])))]
    for h1, h2 in b["proposerSlashings"]:
        for x in (h1, h2):
            out.append(("single", [h1["proposerIndex"]], signing_root(header_root(x), dom(0, x["slot"]))))
    for a1, a2 in b["attesterSlashings"]:
        for a in (a1, a2):
            out.append(("aggregate", a["attestingIndices"],
                        signing_root(att_data_root(a["data"]), dom(1, 32 * a["data"]["target"]["epoch"]))))
    for a in b["attestations"]:
        out.append(("aggregate", a["attestingIndices"],
                    signing_root(att_data_root(a["data"]), dom(1, 32 * a["data"]["target"]["epoch"]))))
    for x in b["voluntaryExits"]:
        out.append(("single", [x["validatorIndex"]],
                    signing_root(merkle([u64(x["epoch"]), u64(x["validatorIndex"])]), dom(4, 32 * x["epoch"]))))
    if not c["skipProposerSignature"]:
        out.append(("single", [b["proposerIndex"]], signing_root(header_root(b), dom(0, b["slot"]))))
    if b["slot"] // 32 >= [f["epoch"] for f in forks if f["name"] == "altair"][0]:
        bits = bytes.fromhex(b["syncAggregate"]["bits"])
        part = [v for i, v in enumerate(c["syncCommittee"]) if (bits[i >> 3] >> (i & 7)) & 1]
        if part:
            out.append(("aggregate", part, signing_root(bytes.fromhex(b["parentRoot"]), dom(7, max(b["slot"], 1) - 1))))
    return out


def produced(c, tmp_path):
    f = tmp_path / "case.json"
    f.write_text(json.dumps(c))
    return json.loads(node("sets", str(f)))


# ---- tests ------------------------------------------------------------------------------------
@pytest.mark.skipif(not os.path.exists(MAINNET_BLOCKS), reason="reference fixture not present")
def test_mainnet_block_roots_chain():
    blocks = json.load(open(MAINNET_BLOCKS))
    got = json.loads(node("roots", MAINNET_BLOCKS))
    for i in range(3):
        assert got[i]["blockRoot"] == blocks[i + 1]["message"]["parent_root"][2:], i
    # phase0 mainnet blocks: randao + attestations + proposer, no sync aggregate
    for g, b in zip(got, blocks):
        assert len(g["sets"]) == 2 + len(b["message"]["body"]["attestations"])


def test_mainnet_fork_digests():
    for version, digest in (("00000000", "b5303f2a"), ("01000000", "afcaaba0"), ("02000000", "4a26c58b")):
        assert node("digest", version, MAINNET_GVR) == digest
        assert merkle([bytes.fromhex(version) + bytes(28), bytes.fromhex(MAINNET_GVR)])[:4].hex() == digest


def test_reference_unit_case_phase0(tmp_path):
    """signatureSets.test.ts:16-81: block + randao + 2 proposer-slashing + 2 attester-slashing
    + 1 attestation + 1 exit signatures (our case has two attestations: 8)."""
    c = make_case(altair_epoch=10)  # phase0 block
    got = produced(c, tmp_path)
    assert len(got) == 1 + 1 + 2 + 2 + 2 + 1
    exp = expected_sets(c)
    assert [(s["type"], s["indices"], s["signingRoot"]) for s in got] == [(t, i, r.hex()) for t, i, r in exp]
    c["skipProposerSignature"] = True
    assert len(produced(c, tmp_path)) == len(got) - 1


def test_altair_sync_aggregate_rules(tmp_path):
    c = make_case()
    got = produced(c, tmp_path)
    exp = expected_sets(c)
    assert got[-1]["type"] == "aggregate" and got[-1]["indices"] == [3, 7, 9, 15]
    assert [(s["type"], s["indices"], s["signingRoot"]) for s in got] == [(t, i, r.hex()) for t, i, r in exp]
    # the attestation targeting epoch 0 signs under phase0's version, the epoch-1 one under altair's
    assert got[6]["signingRoot"] != got[5]["signingRoot"]
    # no participants + infinity signature: no set; no participants + other signature: throws
    inf = "c0" + "00" * 95
    assert len(produced(make_case(sync_bits=[0] * 8, sync_sig=inf), tmp_path)) == len(got) - 1
    assert produced(make_case(sync_bits=[0] * 8), tmp_path) == {"error": "Empty sync committee signature is not infinity"}


@pytest.mark.gpu
def test_block_sets_verify_through_gpu_verifier(tmp_path):
    """Sign the Python-restated roots with interop keys on the device, put the signatures in
    the block, let the JS producers rebuild the sets (indices only) and verify them through
    BlsGpuVerifier: valid; with one set's root swapped: false."""
    from lodestar_amd import build, native
    assert build.build_node(verbose=False), "Node headers missing"
    sks = [int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R for i in range(16)]
    c = make_case()
    exp = expected_sets(c)
    ctx = native.Context()
    agg = [sum(sks[i] for i in idx) % R for _, idx, _ in exp]
    sig = ctx.sign(b"".join(k.to_bytes(32, "big") for k in agg), b"".join(r for _, _, r in exp))
    ctx.close()
    sigs = [sig[96 * i:96 * i + 96].hex() for i in range(len(exp))]
    b = c["block"]
    k = 0
    b["randaoReveal"] = sigs[k]; k += 1  # noqa: E702
    for pair in b["proposerSlashings"]:
        for x in pair:
            x["signature"] = sigs[k]; k += 1  # noqa: E702
    for pair in b["attesterSlashings"]:
        for x in pair:
            x["signature"] = sigs[k]; k += 1  # noqa: E702
    for a in b["attestations"]:
        a["signature"] = sigs[k]; k += 1  # noqa: E702
    for x in b["voluntaryExits"]:
        x["signature"] = sigs[k]; k += 1  # noqa: E702
    b["signature"] = sigs[k]; k += 1  # noqa: E702
    b["syncAggregate"]["signature"] = sigs[k]
    c["secretKeys"] = b"".join(s.to_bytes(32, "big") for s in sks).hex()
    f = tmp_path / "case.json"
    f.write_text(json.dumps(c))
    out = json.loads(node("verify", str(f), timeout=300))
    assert out == {"valid": True, "corrupt": False, "nsets": len(exp)}
