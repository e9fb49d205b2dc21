"""BLS12-381 CPU oracle — TEST INFRASTRUCTURE ONLY.

This module is the checker for the MI355X verifier.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product path (``lodestar_amd``) never does.

It is a plain big-integer restatement of what Lodestar's verify path computes.
The reference repository holds no BLS arithmetic of its own: every call goes
through the un-vendored dependency ``@chainsafe/bls@7.1.1`` ->
``@chainsafe/blst@0.2.4`` -> supranational blst (``yarn.lock:458-473``).
The call sites this file restates are

* ``packages/beacon-node/src/chain/bls/maybeBatch.ts:16-39``
  (``verifySignatureSetsMaybeBatch``: batch >= 2 sets, single verify, empty throws)
* ``packages/beacon-node/src/chain/bls/utils.ts:5-16``  (``PublicKey.aggregate``)
* ``packages/beacon-node/src/chain/bls/multithread/worker.ts:110-116``
  (96-byte uncompressed affine pubkeys, no validation)
* ``packages/state-transition/src/util/interop.ts:19-22`` (interop secret keys)

and the published algorithms the dependency implements:

* ZCash BLS12-381 point serialisation (flags 0x80 compressed / 0x40 infinity /
  0x20 sign = lexicographically largest y).
* RFC 9380 ``BLS12381G2_XMD:SHA-256_SSWU_RO_`` (expand_message_xmd, hash_to_field,
  simplified SWU on the 3-isogenous curve, iso_map §E.3, clear_cofactor via h_eff),
  DST ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`` (IETF BLS sig draft, POP).
* Optimal-ate pairing with loop parameter |x| = 0xd201000000010000 and final
  exponentiation (p^12 - 1) / r.
* blst batch semantics (``verifyMultipleAggregateSignatures``): per-set nonzero
  64-bit random scalar r_i, check prod e(r_i pk_i, H(m_i)) * e(-G1, sum r_i sig_i) == 1,
  infinity signatures skipped, infinity public key -> BLST_PK_IS_INFINITY.

Parity pins (see tests/test_oracle_kat.py):
  * 100 interop pubkeys, ``state-transition/test-cache/interop-pubkeys.json``
    (pins keygen, G1 scalar multiplication and compressed G1 encoding);
  * the interop deposit-0 signature, ``beacon-node/test/e2e/interop/genesisState.test.ts:51-55``
    (pins hash_to_G2, G2 scalar mult, compressed G2 encoding and, through a
    pairing check, the pairing itself).

Pure Python integers: intended for small cases (a pairing costs ~0.1 s).
"""
from __future__ import annotations

import hashlib

# ----------------------------------------------------------------------------
# Parameters
# ----------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # BLS parameter x = -X_ABS
X = -X_ABS
DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# Error codes, numbered as blst's BLST_ERROR enum; INVALID_SIZE is the extra
# code @chainsafe/blst raises for a wrong-length input (multithread.test.ts:100).
BLST_SUCCESS = 0
BLST_BAD_ENCODING = 1
BLST_POINT_NOT_ON_CURVE = 2
BLST_POINT_NOT_IN_GROUP = 3
BLST_AGGR_TYPE_MISMATCH = 4
BLST_VERIFY_FAIL = 5
BLST_PK_IS_INFINITY = 6
BLST_BAD_SCALAR = 7
BLST_INVALID_SIZE = 8
ERROR_NAMES = {
    BLST_BAD_ENCODING: "BLST_BAD_ENCODING",
    BLST_POINT_NOT_ON_CURVE: "BLST_POINT_NOT_ON_CURVE",
    BLST_POINT_NOT_IN_GROUP: "BLST_POINT_NOT_IN_GROUP",
    BLST_AGGR_TYPE_MISMATCH: "BLST_AGGR_TYPE_MISMATCH",
    BLST_VERIFY_FAIL: "BLST_VERIFY_FAIL",
    BLST_PK_IS_INFINITY: "BLST_PK_IS_INFINITY",
    BLST_BAD_SCALAR: "BLST_BAD_SCALAR",
    BLST_INVALID_SIZE: "BLST_INVALID_SIZE",
}


class BlstError(Exception):
    def __init__(self, code: int):
        super().__init__(ERROR_NAMES.get(code, "BLST_ERROR_%d" % code))
        self.code = code


# ----------------------------------------------------------------------------
# Fp
# ----------------------------------------------------------------------------
def inv(a: int) -> int:
    return pow(a, P - 2, P)


def fp_sqrt(a: int):
    """p = 3 mod 4: candidate a^((p+1)/4); None when a is not a square."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


# ----------------------------------------------------------------------------
# Fp2 = Fp[i] / (i^2 + 1), elements as tuples (c0, c1)
# ----------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a0, a1=0):
    return (a0 % P, a1 % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, k: int):
    return (a[0] * k % P, a[1] * k % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * n % P, (-a[1]) * n % P)


def f2_pow(a, e: int):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_sqr(a)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def f2_is_square(a) -> bool:
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """Some square root of a in Fp2 (complex method), or None."""
    a0, a1 = a
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0)
        return None if s is None else (0, s)
    g = fp_sqrt(a0 * a0 + a1 * a1)
    if g is None:
        return None
    inv2 = inv(2)
    d = (a0 + g) * inv2 % P
    x0 = fp_sqrt(d)
    if x0 is None:
        d = (a0 - g) * inv2 % P
        x0 = fp_sqrt(d)
        if x0 is None:
            return None
    x1 = a1 * inv(2 * x0) % P
    r = (x0, x1)
    return r if f2_sqr(r) == (a0 % P, a1 % P) else None


def fp_sgn0(a: int) -> int:
    return a % P % 2


def f2_sgn0(a) -> int:
    """RFC 9380 §4.1 sgn0 for m = 2."""
    sign_0 = a[0] % 2
    zero_0 = a[0] == 0
    sign_1 = a[1] % 2
    return sign_0 | (zero_0 & sign_1)


HALF_P = (P - 1) // 2


def fp_lex_largest(a: int) -> bool:
    return a > HALF_P


def f2_lex_largest(a) -> bool:
    """ZCash sign bit for Fp2: compare c1 first, c0 when c1 == 0."""
    if a[1] != 0:
        return a[1] > HALF_P
    return a[0] > HALF_P


XI = (1, 1)  # non-residue 1 + i: Fp6 = Fp2[v]/(v^3 - XI), w^6 = XI

# ----------------------------------------------------------------------------
# Fp12 flat over w: f = sum_{j<6} c_j w^j, c_j in Fp2, w^6 = XI.
# (Tower view: Fp12 = Fp6[w]/(w^2 - v), Fp6 = Fp2[v]/(v^3 - XI): c_{2k} is the
# v^k coefficient of the "a" half, c_{2k+1} of the "b" half.)
# ----------------------------------------------------------------------------
F12_ONE = (F2_ONE,) + (F2_ZERO,) * 5


def f12_mul(a, b):
    acc = [(0, 0)] * 11
    for i in range(6):
        ai = a[i]
        if ai == (0, 0):
            continue
        for j in range(6):
            bj = b[j]
            if bj == (0, 0):
                continue
            acc[i + j] = f2_add(acc[i + j], f2_mul(ai, bj))
    out = list(acc[:6])
    for k in range(6, 11):
        out[k - 6] = f2_add(out[k - 6], f2_mul(acc[k], XI))
    return tuple(out)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    """a^(p^6): w -> -w."""
    return tuple(c if j % 2 == 0 else f2_neg(c) for j, c in enumerate(a))


# Frobenius: (sum c_j w^j)^p = sum conj(c_j) * GAMMA[j] * w^j, GAMMA[j] = XI^(j(p-1)/6)
FROB_GAMMA = [f2_pow(XI, j * (P - 1) // 6) for j in range(6)]


def f12_frob(a):
    return tuple(f2_mul(f2_conj(a[j]), FROB_GAMMA[j]) for j in range(6))


def f12_inv(a):
    # a^-1 = a^(p^12 - 2); only used on small paths (tests)
    return f12_pow(a, P**12 - 2)


def f12_pow(a, e: int):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_sqr(a)
        e >>= 1
    return r


def f12_eq(a, b):
    return tuple(a) == tuple(b)


def f12_to_tower_list(a):
    """Serialisation order used across the repo: tower coefficients
    [a.c0, a.c1, a.c2, b.c0, b.c1, b.c2] (each Fp2 as (re, im)) — i.e. flat
    indices [0, 2, 4, 1, 3, 5]."""
    out = []
    for j in (0, 2, 4, 1, 3, 5):
        out.extend(a[j])
    return out


# ----------------------------------------------------------------------------
# Curves: affine points as (x, y) or None for infinity.
# E1: y^2 = x^3 + 4 over Fp.  E2: y^2 = x^3 + 4(1+i) over Fp2.
# ----------------------------------------------------------------------------
B1 = 4
B2 = (4, 4)

G1 = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2 = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)


# --- generic affine group law, parameterised by field ops -------------------
class _Field:
    def __init__(self, add, sub, mul, sqr, inv_, neg, zero, one, muls):
        self.add, self.sub, self.mul, self.sqr = add, sub, mul, sqr
        self.inv, self.neg, self.zero, self.one, self.muls = inv_, neg, zero, one, muls


FP = _Field(
    lambda a, b: (a + b) % P,
    lambda a, b: (a - b) % P,
    lambda a, b: a * b % P,
    lambda a: a * a % P,
    inv,
    lambda a: (-a) % P,
    0,
    1,
    lambda a, k: a * k % P,
)
FP2 = _Field(f2_add, f2_sub, f2_mul, f2_sqr, f2_inv, f2_neg, F2_ZERO, F2_ONE, f2_muls)


def _add(F, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if y1 == y2 and y1 != F.zero:
            lam = F.mul(F.muls(F.sqr(x1), 3), F.inv(F.muls(y1, 2)))
        else:
            return None
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.sqr(lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def _neg(F, p1):
    return None if p1 is None else (p1[0], F.neg(p1[1]))


def _mul(F, p1, k: int):
    if k < 0:
        return _mul(F, _neg(F, p1), -k)
    acc = None
    while k:
        if k & 1:
            acc = _add(F, acc, p1)
        p1 = _add(F, p1, p1)
        k >>= 1
    return acc


def g1_add(a, b):
    return _add(FP, a, b)


def g1_neg(a):
    return _neg(FP, a)


def g1_mul(a, k):
    return _mul(FP, a, k)


def g2_add(a, b):
    return _add(FP2, a, b)


def g2_neg(a):
    return _neg(FP2, a)


def g2_mul(a, k):
    return _mul(FP2, a, k)


def g1_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g1_in_group(pt) -> bool:
    return g1_on_curve(pt) and g1_mul(pt, R) is None


def g2_in_group(pt) -> bool:
    return g2_on_curve(pt) and g2_mul(pt, R) is None


# --- psi endomorphism on E2 (untwist-Frobenius-twist) -----------------------
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    x, y = pt
    return (f2_mul(f2_conj(x), PSI_CX), f2_mul(f2_conj(y), PSI_CY))


# ----------------------------------------------------------------------------
# ZCash serialisation
# ----------------------------------------------------------------------------
def _i2b(v: int, n: int) -> bytes:
    return v.to_bytes(n, "big")


def g1_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(_i2b(x, 48))
    b[0] |= 0x80 | (0x20 if fp_lex_largest(y) else 0)
    return bytes(b)


def g1_serialize(pt) -> bytes:
    """96-byte uncompressed x || y (PublicKey.toBytes(PointFormat.uncompressed))."""
    if pt is None:
        return bytes([0x40]) + bytes(95)
    return _i2b(pt[0], 48) + _i2b(pt[1], 48)


def g1_decompress(b: bytes):
    """Compressed 48-byte G1 -> affine point, raising BlstError like blst_p1_uncompress."""
    if len(b) != 48:
        raise BlstError(BLST_INVALID_SIZE)
    flags = b[0]
    if not flags & 0x80:
        raise BlstError(BLST_BAD_ENCODING)
    if flags & 0x40:
        if (flags & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x = int.from_bytes(bytes([flags & 0x1F]) + b[1:], "big")
    if x >= P:
        raise BlstError(BLST_BAD_ENCODING)
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if fp_lex_largest(y) != bool(flags & 0x20):
        y = (-y) % P
    if x == 0:  # (0, +-2): on the curve, order 3 (blst POINTonE1_Uncompress_Z)
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return (x, y)


def g1_deserialize(b: bytes):
    """96-byte G1 record, no subgroup check (worker.ts:112 trusts pubkeys), decoded as
    blst's POINTonE1_Deserialize_Z does for PublicKey.fromBytes of 96 bytes:
    top bits 000 -> big-endian x || y; 0x80 -> the first 48 bytes compressed;
    0x40 alone -> infinity iff all other bits are zero; otherwise BAD_ENCODING."""
    if len(b) != 96:
        raise BlstError(BLST_INVALID_SIZE)
    if b[0] & 0x80:
        return g1_decompress(bytes(b[:48]))
    if b[0] & 0x40:
        if (b[0] & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    if b[0] & 0x20:
        raise BlstError(BLST_BAD_ENCODING)
    x = int.from_bytes(b[:48], "big")
    y = int.from_bytes(b[48:], "big")
    if x >= P or y >= P:
        raise BlstError(BLST_BAD_ENCODING)
    pt = (x, y)
    if not g1_on_curve(pt):
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if x == 0:
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


def g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(_i2b(x[1], 48) + _i2b(x[0], 48))
    b[0] |= 0x80 | (0x20 if f2_lex_largest(y) else 0)
    return bytes(b)


def g2_serialize(pt) -> bytes:
    """192-byte uncompressed: x.c1 || x.c0 || y.c1 || y.c0."""
    if pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = pt
    return _i2b(x[1], 48) + _i2b(x[0], 48) + _i2b(y[1], 48) + _i2b(y[0], 48)


def g2_decompress(b: bytes):
    """Compressed 96-byte G2 -> affine point or None (infinity); raises BlstError.
    Mirrors blst_p2_uncompress (no subgroup check; see signature_from_bytes)."""
    if len(b) != 96:
        raise BlstError(BLST_INVALID_SIZE)
    flags = b[0]
    if not flags & 0x80:
        raise BlstError(BLST_BAD_ENCODING)
    if flags & 0x40:
        if (flags & 0x3F) == 0 and not any(b[1:]):
            return None
        raise BlstError(BLST_BAD_ENCODING)
    x1 = int.from_bytes(bytes([flags & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        raise BlstError(BLST_BAD_ENCODING)
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise BlstError(BLST_POINT_NOT_ON_CURVE)
    if f2_lex_largest(y) != bool(flags & 0x20):
        y = f2_neg(y)
    return (x, y)


def signature_from_bytes(b: bytes, validate: bool = True):
    """bls.Signature.fromBytes(bytes, CoordType.affine, validate=true)
    (maybeBatch.ts:23,36): 96-byte compressed only on this path; subgroup
    check when validate."""
    pt = g2_decompress(b)
    if validate and pt is not None and not g2_in_group(pt):
        raise BlstError(BLST_POINT_NOT_IN_GROUP)
    return pt


# ----------------------------------------------------------------------------
# Keys (interop keygen: state-transition/src/util/interop.ts:19-22)
# ----------------------------------------------------------------------------
def interop_secret_key(index: int) -> int:
    d = hashlib.sha256(index.to_bytes(32, "little")).digest()
    return int.from_bytes(d, "little") % R


def sk_to_pk(sk: int):
    return g1_mul(G1, sk)


def pubkey_aggregate(pks):
    """bls.PublicKey.aggregate (utils.ts:11) — EMPTY_AGGREGATE_ARRAY on []."""
    if len(pks) == 0:
        raise ValueError("EMPTY_AGGREGATE_ARRAY")
    acc = None
    for pk in pks:
        acc = g1_add(acc, pk)
    return acc


# ----------------------------------------------------------------------------
# hash_to_G2: RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_
# ----------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in = 32
    r_in = 64
    ell = (len_in_bytes + b_in - 1) // b_in
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(r_in) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    b = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(2, ell + 1):
        prev = bytes(x ^ y for x, y in zip(b0, b[-1]))
        b.append(hashlib.sha256(prev + bytes([i]) + dst_prime).digest())
    return b"".join(b)[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, dst: bytes, count: int = 2):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = []
        for j in range(2):
            off = L * (j + i * 2)
            e.append(int.from_bytes(ub[off:off + L], "big") % P)
        out.append((e[0], e[1]))
    return out


# E2': y^2 = x^3 + A' x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)

_ISO = {
    "xnum": [
        (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
         0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
        (0,
         0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
        (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
         0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
        (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1,
         0),
    ],
    "xden": [
        (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
        (0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
        (1, 0),
    ],
    "ynum": [
        (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
         0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
        (0,
         0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
        (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
         0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
        (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10,
         0),
    ],
    "yden": [
        (0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
         0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
        (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
        (0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
        (1, 0),
    ],
}
ISO_CONSTANTS = _ISO


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map_g2(pt):
    """3-isogeny E2' -> E2 (RFC 9380 Appendix E.3)."""
    if pt is None:
        return None
    x, y = pt
    xd = _poly(_ISO["xden"], x)
    yd = _poly(_ISO["yden"], x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    xo = f2_mul(_poly(_ISO["xnum"], x), f2_inv(xd))
    yo = f2_mul(y, f2_mul(_poly(_ISO["ynum"], x), f2_inv(yd)))
    return (xo, yo)


def sswu_g2(u):
    """RFC 9380 §6.6.2 simplified SWU onto E2' (returns affine point on E2')."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    den = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(den):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(den)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x2 = f2_mul(zu2, x1)
        gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(A, x2)), B)
        x, y = x2, f2_sqrt(gx2)
    assert y is not None
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def map_to_curve_g2(u):
    return iso_map_g2(sswu_g2(u))


H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551


def clear_cofactor_g2(pt):
    """RFC 9380 Appendix G.4 (psi-based), equal to [h_eff] pt."""
    t1 = g2_mul(pt, X)
    t2 = g2_psi(pt)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    t3 = g2_add(t3, g2_neg(t2))
    t2 = g2_add(t1, t2)
    t2 = g2_mul(t2, X)
    t3 = g2_add(t3, t2)
    t3 = g2_add(t3, g2_neg(t1))
    return g2_add(t3, g2_neg(pt))


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    q = g2_add(map_to_curve_g2(u0), map_to_curve_g2(u1))
    return clear_cofactor_g2(q)


def sign(sk: int, msg: bytes, dst: bytes = DST_POP):
    return g2_mul(hash_to_g2(msg, dst), sk)


# ----------------------------------------------------------------------------
# Pairing (textbook affine Miller loop on the twist, lines embedded in Fp12)
# ----------------------------------------------------------------------------
def _line_to_f12(lam, xq, yq, xp, yp):
    """Line through T=(xq,yq) with slope lam (twist coords) evaluated at P,
    scaled by w^3: (lam*xq - yq) + (-lam*xp) w^2 + yp w^3."""
    c0 = f2_sub(f2_mul(lam, xq), yq)
    c2 = f2_muls(lam, (-xp) % P)
    c3 = (yp % P, 0)
    return (c0, F2_ZERO, c2, c3, F2_ZERO, F2_ZERO)


def _vertical_free_miller(p1, q2):
    xp, yp = p1
    t = q2
    f = F12_ONE
    bits = bin(X_ABS)[3:]
    for bit in bits:
        # doubling step
        xt, yt = t
        lam = f2_mul(f2_muls(f2_sqr(xt), 3), f2_inv(f2_muls(yt, 2)))
        f = f12_mul(f12_sqr(f), _line_to_f12(lam, xt, yt, xp, yp))
        x3 = f2_sub(f2_sqr(lam), f2_muls(xt, 2))
        y3 = f2_sub(f2_mul(lam, f2_sub(xt, x3)), yt)
        t = (x3, y3)
        if bit == "1":
            xt, yt = t
            xq, yq = q2
            lam = f2_mul(f2_sub(yt, yq), f2_inv(f2_sub(xt, xq)))
            f = f12_mul(f, _line_to_f12(lam, xt, yt, xp, yp))
            x3 = f2_sub(f2_sub(f2_sqr(lam), xt), xq)
            y3 = f2_sub(f2_mul(lam, f2_sub(xt, x3)), yt)
            t = (x3, y3)
    return f


def miller_loop(p1, q2):
    """f_{x,Q}(P) for x < 0 (conjugated), P in G1, Q in G2 (both affine)."""
    if p1 is None or q2 is None:
        return F12_ONE
    return f12_conj(_vertical_free_miller(p1, q2))


HARD_EXP = (P**4 - P**2 + 1) // R


def final_exp(f):
    # easy part: f^(p^6 - 1) (p^2 + 1)
    f = f12_mul(f12_conj(f), f12_inv_fast(f))
    f = f12_mul(f12_frob(f12_frob(f)), f)
    # hard part
    return f12_pow(f, HARD_EXP)


def f12_inv_fast(a):
    """Inverse via norm to Fp6 (tower view) — a = A + B w, a^-1 = (A - B w)/(A^2 - B^2 v)."""
    A = (a[0], a[2], a[4])
    B = (a[1], a[3], a[5])

    def f6_mul(x, y):
        # Fp6 = Fp2[v]/(v^3 - XI)
        c = [F2_ZERO] * 5
        for i in range(3):
            for j in range(3):
                c[i + j] = f2_add(c[i + j], f2_mul(x[i], y[j]))
        return (f2_add(c[0], f2_mul(c[3], XI)), f2_add(c[1], f2_mul(c[4], XI)), c[2])

    def f6_mulv(x):
        return (f2_mul(x[2], XI), x[0], x[1])

    def f6_inv(x):
        a0, a1, a2 = x
        t0 = f2_sub(f2_sqr(a0), f2_mul(f2_mul(a1, a2), XI))
        t1 = f2_sub(f2_mul(f2_sqr(a2), XI), f2_mul(a0, a1))
        t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
        d = f2_add(f2_mul(a0, t0), f2_mul(f2_add(f2_mul(a2, t1), f2_mul(a1, t2)), XI))
        di = f2_inv(d)
        return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))

    AA = f6_mul(A, A)
    BB = f6_mulv(f6_mul(B, B))
    n = tuple(f2_sub(AA[i], BB[i]) for i in range(3))
    ni = f6_inv(n)
    A2 = f6_mul(A, ni)
    B2_ = f6_mul(B, ni)
    B2_ = tuple(f2_neg(c) for c in B2_)
    return (A2[0], B2_[0], A2[1], B2_[1], A2[2], B2_[2])


def pairing(p1, q2):
    return final_exp(miller_loop(p1, q2))


# ----------------------------------------------------------------------------
# Verify semantics (blst / @chainsafe/blst, called from maybeBatch.ts)
# ----------------------------------------------------------------------------
NEG_G1 = g1_neg(G1)


def core_verify(pk, msg: bytes, sig) -> bool:
    """Signature.verify(pk, msg): e(pk, H(m)) == e(G1, sig) (maybeBatch.ts:34-38)."""
    if pk is None:
        return False  # BLST_PK_IS_INFINITY -> verify returns false (unpinned; blst semantics)
    h = hash_to_g2(msg)
    f = f12_mul(miller_loop(pk, h), miller_loop(NEG_G1, sig))
    return final_exp(f) == F12_ONE


def verify_multiple(sets, scalars):
    """verifyMultipleAggregateSignatures: sets = [(pk_affine, msg, sig_affine)],
    scalars = nonzero 64-bit ints (injected for determinism)."""
    f = F12_ONE
    s_acc = None
    for (pk, msg, sig), r in zip(sets, scalars):
        assert 0 < r < 2**64
        if sig is not None:
            s_acc = g2_add(s_acc, g2_mul(sig, r))
        if pk is None:
            raise BlstError(BLST_PK_IS_INFINITY)
        h = hash_to_g2(msg)
        f = f12_mul(f, miller_loop(g1_mul(pk, r), h))
    if s_acc is not None:
        f = f12_mul(f, miller_loop(NEG_G1, s_acc))
    return final_exp(f) == F12_ONE


def verify_signature_sets_maybe_batch(sets, scalars=None):
    """maybeBatch.ts:16-39.  sets = [(pk_affine, msg32, sig_bytes)].
    Returns bool or raises BlstError / ValueError (empty)."""
    if len(sets) >= 2:
        parsed = [(pk, msg, signature_from_bytes(sig, True)) for pk, msg, sig in sets]
        if scalars is None:
            import secrets
            scalars = [secrets.randbits(64) or 1 for _ in sets]
        return verify_multiple(parsed, scalars)
    if len(sets) == 0:
        raise ValueError("Empty signature set")
    for pk, msg, sig in sets:
        s = signature_from_bytes(sig, True)
        if not core_verify(pk, msg, s):
            return False
    return True


def chunkify_maximize_chunk_size(arr, min_per_chunk: int):
    """multithread/utils.ts:4-19."""
    chunk_count = len(arr) // min_per_chunk
    if chunk_count <= 1:
        return [list(arr)]
    per_chunk = -(-len(arr) // chunk_count)
    return [list(arr[i:i + per_chunk]) for i in range(0, len(arr), per_chunk)]


# ----------------------------------------------------------------------------
# deposit-time key validation, op-pool signature aggregation
# ----------------------------------------------------------------------------
def pubkey_validate(b: bytes) -> int:
    """bls.PublicKey.fromBytes(pubkey, CoordType.affine, validate=true)
    (state-transition/src/block/processDeposit.ts:64): ZCash decode, then blst's
    key validation — infinity -> BLST_PK_IS_INFINITY, outside G1 ->
    BLST_POINT_NOT_IN_GROUP.  Returns 0 or the BLST code."""
    try:
        pt = g1_decompress(b)
    except BlstError as e:
        return e.code
    if pt is None:
        return BLST_PK_IS_INFINITY
    if not g1_in_group(pt):
        return BLST_POINT_NOT_IN_GROUP
    return 0


def signatures_aggregate(sigs):
    """bls.Signature.aggregate(sigs.map(s => Signature.fromBytes(s, undefined, true)))
    (chain/opPools/attestationPool.ts:184-187, aggregatedAttestationPool.ts:319-321,
    syncCommitteeMessagePool.ts:126-129, syncContributionAndProofPool.ts:181-185).
    Returns (0, compressed 96 B) or (code, None): the first failing signature's
    BLST code, 20 (EMPTY_AGGREGATE_ARRAY) for [].  An infinity signature decodes
    and adds nothing (dependency-defined; unpinned here)."""
    if len(sigs) == 0:
        return 20, None
    acc = None
    for s in sigs:
        try:
            acc = g2_add(acc, signature_from_bytes(s, True))
        except BlstError as e:
            return e.code, None
    return 0, g2_compress(acc)


def deposit_valid(pk48: bytes, msg32: bytes, sig96: bytes) -> bool:
    """processDeposit.ts:62-70: key validated, signature validated and verified;
    any BLS error counts as invalid (the catch-all returns)."""
    if pubkey_validate(pk48) != 0:
        return False
    try:
        sig = signature_from_bytes(sig96, True)
    except BlstError:
        return False
    if sig is None:
        return False
    return core_verify(g1_decompress(pk48), msg32, sig)
