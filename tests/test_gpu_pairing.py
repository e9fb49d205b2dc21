"""GPU: the device's per-set pairing values pinned to the oracle with injected randomizers.

bgv_debug_prepare runs a call's verify kernels (bulk: k_prep + k_miller; latency: k_prep_a +
the wide / team kernels) with set i's randomizer the i-th nonzero splitmix64 word of the seed
and returns every set's Miller value f_i.  tests/golden/pairing.json holds, for the same seed,
the oracle's e(r_i pk_i, H(m_i)) and its textbook Miller value m_i.  Checked on both paths:
  * final_exp(f_i) == e_i with the oracle's final exponentiation on the host, for every set
    (the pure-Python exponentiation takes ~1 s each);
  * on the device, bgv_final_verify over the committed partial product f_i * conj(m_i) is 1
    for every set (final_exp(conj(m)) = e^-1), and 0 for f_i * conj(m_j), j != i.
Bit-exact integer work.  Reference: packages/beacon-node/src/chain/bls/maybeBatch.ts:18-25.
"""
import json
import os

import pytest

from tests.test_pairing_golden import GOLD, f12_from_bytes

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def conj_bytes(b):
    """conj(f) = f^(p^6): negate the b half (tower coefficients 6..11)."""
    P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
    out = bytearray(b[:288])
    for i in range(6, 12):
        v = int.from_bytes(b[48 * i:48 * i + 48], "big")
        out += ((P - v) % P).to_bytes(48, "big")
    return bytes(out)


@pytest.fixture(scope="module")
def ctx():
    from lodestar_amd import native
    c = native.Context()
    keys = json.load(open(os.path.join(HERE, "golden", "keys.json")))
    c.pubkeys_put(0, b"".join(bytes.fromhex(k) for k in keys["pk_compressed"]), native.PK_COMPRESSED)
    yield c
    c.close()


def _sets():
    from lodestar_amd import native
    return [native.SetSpec(bytes.fromhex(s["msg"]), bytes.fromhex(s["sig"]), pk_indices=s["pk_indices"])
            for s in GOLD["sets"]]


@pytest.mark.parametrize("path", ["bulk", "latency"])
def test_device_pairing_values(ctx, path):
    from lodestar_amd import native
    from oracle import bls12381 as o
    p = native.PATH_BULK if path == "bulk" else native.PATH_LATENCY
    out = ctx.debug_prepare(_sets(), p, seed=GOLD["seed"])
    assert len(out) == len(GOLD["sets"])
    for (_, f, ss, ps), s in zip(out, GOLD["sets"]):
        assert ss == 0 and ps == 0
        assert ctx.final_verify([f, conj_bytes(bytes.fromhex(s["miller"]))]), s["pk_indices"]
    # negative controls: another set's pairing value
    for i in (0, 9):
        j = (i + 1) % len(out)
        assert not ctx.final_verify([out[i][1], conj_bytes(bytes.fromhex(GOLD["sets"][j]["miller"]))])
    # host final exponentiation (oracle) of every device value, independent of the device's
    for i in range(len(out)):
        assert o.final_exp(f12_from_bytes(out[i][1])) == f12_from_bytes(bytes.fromhex(GOLD["sets"][i]["gt"])), i
