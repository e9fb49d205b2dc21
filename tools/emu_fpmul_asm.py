"""Check tools/gen_fpmul_asm.py's output without a GPU: a Python emulation of the generated
bgv_fpmul_x / bgv_fpsqr_x instruction streams against fp_mul_body / fp_sqr_body's row-wise
Montgomery product (bls_field.h), limb for limb, with overflow checks on every 64-bit result.

    python tools/emu_fpmul_asm.py [n]
"""
import os
import random
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "experimental", "bgv_fpmul_asm.h")
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
N0, M = 0xffcfffd, (1 << 28) - 1


def routine(src, name):
    body, on = [], False
    for ln in re.findall(r'"  (.*)\\n"', src):
        if ln == name + ":":
            on = True
            continue
        if on:
            if ln.startswith("s_setpc"):
                return body
            body.append(ln)
    raise KeyError(name)


def run(body, a, b):
    V, S = {}, {}
    for i in range(14):
        V[i], V[14 + i] = a[i], b[i]
    written = set()

    def g64(r):
        lo = int(re.match(r"v\[(\d+):(\d+)\]", r).group(1))
        return V[lo] | (V[lo + 1] << 32)

    def s64(r, val):
        assert 0 <= val < 1 << 64, "64-bit overflow"
        lo = int(re.match(r"v\[(\d+):(\d+)\]", r).group(1))
        V[lo], V[lo + 1] = val & 0xFFFFFFFF, val >> 32
        written.update((lo, lo + 1))

    def g32(x):
        if x.startswith("v"):
            return V[int(x[1:])]
        if x.startswith("s"):
            return S[int(x[1:])]
        return int(x, 0)

    def s32(d, val):
        V[int(d[1:])] = val & 0xFFFFFFFF
        written.add(int(d[1:]))

    for ln in body:
        op, rest = ln.split(None, 1)
        o = [x.strip() for x in rest.split(",")]
        if op == "s_mov_b32":
            S[int(o[0][1:])] = int(o[1], 0)
        elif op == "v_mad_u64_u32":
            s64(o[0], g32(o[2]) * g32(o[3]) + (0 if o[4] == "0" else g64(o[4])))
        elif op == "v_lshl_add_u64":
            s64(o[0], (g64(o[1]) << int(o[2])) + g64(o[3]))
        elif op == "v_mul_lo_u32":
            s32(o[0], g32(o[1]) * g32(o[2]))
        elif op == "v_and_b32_e32":
            s32(o[0], int(o[1], 0) & g32(o[2]))
        elif op == "v_lshrrev_b64":
            s64(o[0], g64(o[2]) >> int(o[1]))
        elif op == "v_mov_b32_e32":
            s32(o[0], g32(o[1]))
        else:
            raise SystemExit("unknown op " + op)
    assert not any(14 <= r < 28 for r in written), "b clobbered"
    assert all(r < 62 for r in written), "write outside the clobber set"
    return [V[i] for i in range(14)]


def ref(a, b):
    pl = [(P >> (28 * i)) & M for i in range(14)]
    t = [0] * 14
    for i in range(14):
        for j in range(14):
            t[j] += a[i] * b[j]
        m = ((t[0] & 0xFFFFFFFF) * N0) & M
        for j in range(14):
            t[j] += m * pl[j]
        c = t[0] >> 28
        t = t[1:] + [0]
        t[0] += c
    r = []
    for j in range(13):
        r.append(t[j] & M)
        t[j + 1] += t[j] >> 28
    r.append(t[13] & 0xFFFFFFFF)
    return r


def main(n=300):
    src = open(SRC).read()
    mul, sqr = routine(src, "bgv_fpmul_x"), routine(src, "bgv_fpsqr_x")
    rng = random.Random(1)
    for k in range(n):
        if k % 3 == 0:  # operand limbs at their bounds (fp_mul_l accepts limbs < 2^29)
            a = [(1 << 29) - 1 - rng.randrange(4) for _ in range(14)]
            b = [(1 << 29) - 1 - rng.randrange(4) for _ in range(14)]
        else:
            a = [rng.randrange(1 << 29) for _ in range(14)]
            b = [rng.randrange(1 << 29) for _ in range(14)]
        a[13], b[13] = rng.randrange(1 << 19), rng.randrange(1 << 19)
        assert run(mul, a, b) == ref(a, b), "bgv_fpmul_x"
        assert run(sqr, a, [0] * 14) == ref(a, a), "bgv_fpsqr_x"
    print("generated asm == fp_mul_body / fp_sqr_body on %d operand pairs" % n)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
