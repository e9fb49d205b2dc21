"""Generate tools/experimental/bgv_fpmul_asm.h (an experiment kept out of the product library): the 28-bit-limb Montgomery product and square as
hand-scheduled gfx950 subroutines with a register contract of their own.

    python tools/gen_fpmul_asm.py

Why (tools/ubench_prod.hip, profiles/r04/ubench_prod.jsonl): the compiler's out-of-line
fp_mul_l costs ~2,850 SIMD cycles per product at one wave per SIMD, the same body inlined
~2,080.  The difference is the ABI call: argument moves, a full s_waitcnt at entry, and a
callee-saved/caller-saved split that leaves the caller only 112 VGPRs + 224 AGPRs across a
call (the verify kernels' spills).  Inlining every product is no way out: the Miller step's
loop body grows to ~400 KB and runs slower (instruction cache; profiles/r04/inline_ab/).

These routines take a = v[0:13], b = v[14:27] and return the product in v[0:13]; they clobber
v[28:61] and s[44:63] only (s[62:63] is the return address), so everything else the caller
holds stays in registers across the call, and the inline-asm call site waits only for its own
operands.  The arithmetic is exactly fp_mul_body / fp_sqr_body's (bls_field.h): the same
Montgomery digits m_i, the same integer (a b + m p) / 2^392, the same limb normalisation
(limbs 0..12 masked to 28 bits, limb 13 the rest), so results are bit-identical
(tests/test_gpu_r04.py::test_asm_products_match).

Schedule: product scanning (columns), each column's products split over two accumulator
chains, list-scheduled for one wave per SIMD (one VALU issue per 4 cycles, 64-bit results
assumed ready 12 cycles after issue) with the critical path (the Montgomery digit chain) first.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "experimental", "bgv_fpmul_asm.h")

P = [0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2, 0xf38512b, 0x4774b84, 0x4bacd76,
     0xba7b643, 0xe69a4b1, 0x1ea397f, 0x001a011]
N0 = 0xffcfffd
NL = 14
MASK = 0xfffffff
S_P = 44       # s44..s57: p limbs
S_N0 = 58
S_CARRY = 60   # s[60:61]: the mads' unused carry-out
S_RET = 62     # s[62:63]: return address
V_A, V_B = 0, 14
V_M = 28       # v28..v41: Montgomery digits (product) / doubled limbs (square)
V_POOL = list(range(42, 62, 2))  # 10 accumulator pairs
LAT64, LAT32, ISSUE = 12, 8, 4


class Ins:
    __slots__ = ("op", "dst", "srcs", "lat", "fmt", "prio", "users", "ready", "done", "idx")

    def __init__(self, op, dst, srcs, fmt, lat):
        self.op, self.dst, self.srcs, self.fmt, self.lat = op, dst, srcs, fmt, lat
        self.users = []


def build(square):
    """The column DAG.  Virtual registers: ('acc', n) 64-bit, ('m', i), ('d', i) 32-bit,
    physical ('a', i) / ('b', i) inputs, ('r', i) outputs."""
    ins = []
    defs = {}
    nacc = [0]

    def new_acc():
        nacc[0] += 1
        return ("acc", nacc[0])

    def emit(op, dst, srcs, fmt, lat):
        i = Ins(op, dst, srcs, fmt, lat)
        i.idx = len(ins)
        ins.append(i)
        if dst is not None:
            defs[dst] = i
        return i

    def terms(k):
        """(product terms, diagonal term): the square's cross products a_i a_j (i < j) are
        summed once and doubled by the combine (shift 1), its diagonal a_{k/2}^2 added."""
        out, diag = [], None
        if square:
            for i in range(NL):
                j = k - i
                if j <= i or j >= NL:
                    continue
                out.append((("a", i), ("a", j)))
            if k % 2 == 0 and k // 2 < NL:
                diag = (("a", k // 2), ("a", k // 2))
        else:
            for i in range(NL):
                j = k - i
                if 0 <= j < NL:
                    out.append((("a", i), ("b", j)))
        return out, diag

    def chain(terms_, nch):
        chains = [None] * nch
        for n, (x, y) in enumerate(terms_):
            c = n % nch
            d = new_acc()
            src = [x, y] + ([chains[c]] if chains[c] else [])
            fmt = "v_mad_u64_u32 {d}, s[%d:%d], {s0}, {s1}, " % (S_CARRY, S_CARRY + 1) + ("{s2}" if chains[c] else "0")
            emit("mad", d, src, fmt, LAT64)
            chains[c] = d
        return [c for c in chains if c]

    def sum64(parts, shift_first=False):
        """parts[0] << (1 if shift_first) + the rest"""
        while len(parts) > 1:
            d = new_acc()
            sh = 1 if shift_first else 0
            emit("add64", d, [parts[0], parts[1]], "v_lshl_add_u64 {d}, {s0}, %d, {s1}" % sh, LAT64)
            parts = [d] + parts[2:]
            shift_first = False
        return parts[0]

    carry = None
    for k in range(2 * NL - 1):
        prods, diag = terms(k)
        # reduction terms m_i p_j (i < k), older digits first (m_{k-1} p_1 last)
        red = [(("m", i), ("p", k - i)) for i in range(NL) if i < min(k, NL) and 0 <= k - i < NL]
        if square:
            cross = chain(prods, 1)
            rest = chain(([diag] if diag else []) + red, 2) + ([carry] if carry else [])
            if cross:
                x = sum64(cross)
                acc = sum64([x] + rest, shift_first=True) if rest else None
                if acc is None:  # only cross terms (cannot happen for k >= 1 with a carry)
                    acc = new_acc()
                    emit("add64", acc, [x, x], "v_lshl_add_u64 {d}, {s0}, 0, {s1}", LAT64)
            else:
                acc = sum64(rest)
        else:
            acc = sum64(chain(prods + red, 2) + ([carry] if carry else []))
        if k < NL:
            mtmp = ("mt", k)
            emit("mullo", mtmp, [acc], "v_mul_lo_u32 {d}, {s0l}, s%d" % S_N0, LAT32)
            emit("and", ("m", k), [mtmp], "v_and_b32_e32 {d}, 0x%x, {s0}" % MASK, LAT32)
            d = new_acc()
            emit("mad", d, [("m", k), ("p", 0), acc],
                 "v_mad_u64_u32 {d}, s[%d:%d], {s0}, {s1}, {s2}" % (S_CARRY, S_CARRY + 1), LAT64)
            acc = d
        else:
            emit("and", ("r", k - NL), [acc], "v_and_b32_e32 {d}, 0x%x, {s0l}" % MASK, LAT32)
        c = new_acc()
        emit("shr", c, [acc], "v_lshrrev_b64 {d}, 28, {s0}", LAT64)
        carry = c
    emit("top", ("r", NL - 1), [carry], "v_mov_b32_e32 {d}, {s0l}", LAT32)
    return ins, defs


def schedule(ins, defs):
    for i in ins:
        for s in i.srcs:
            if s in defs:
                defs[s].users.append(i)
    for i in reversed(ins):  # longest latency path to the end
        i.prio = i.lat + max((u.prio for u in i.users), default=0)
    npred = {i.idx: sum(1 for s in i.srcs if s in defs) for i in ins}
    ready_at = {i.idx: 0 for i in ins}
    avail = [i for i in ins if npred[i.idx] == 0]
    order, t = [], 0
    live_acc = set()
    while avail:
        cand = [i for i in avail if ready_at[i.idx] <= t]
        if not cand:
            t = min(ready_at[i.idx] for i in avail)
            continue

        def opens(i):  # a mad that starts a new accumulator chain (register pressure)
            return i.op == "mad" and not any(s[0] == "acc" for s in i.srcs)
        if len(live_acc) >= len(V_POOL) - 1:
            ok = [i for i in cand if not opens(i)]
            if not ok:  # wait for a chain to advance rather than open another
                later = [i for i in avail if not opens(i)]
                t = min(ready_at[i.idx] for i in later)
                continue
            cand = ok
        pick = max(cand, key=lambda i: (i.prio, -i.idx))
        avail.remove(pick)
        order.append(pick)
        for s in pick.srcs:
            if s[0] == "acc" and all(u in order for u in defs[s].users):
                live_acc.discard(s)
        if pick.dst and pick.dst[0] == "acc":
            live_acc.add(pick.dst)
        for u in pick.users:
            npred[u.idx] -= 1
            ready_at[u.idx] = max(ready_at[u.idx], t + pick.lat)
            if npred[u.idx] == 0:
                avail.append(u)
        t += ISSUE
    assert len(order) == len(ins)
    return order, t


def allocate(order, defs):
    """Linear scan over the accumulator pairs; m / d / outputs at fixed homes."""
    last = {}
    for n, i in enumerate(order):
        for s in i.srcs:
            last[s] = n
    free = list(V_POOL)
    phys = {}
    text = []
    for n, i in enumerate(order):
        def reg(v, lo=False):
            kind, x = v
            if kind == "a":
                return "v%d" % (V_A + x)
            if kind == "b":
                return "v%d" % (V_B + x)
            if kind == "p":
                return "s%d" % (S_P + x)
            if kind == "m":
                return "v%d" % (V_M + x)
            if kind == "mt":
                return "v%d" % (V_M + x)
            if kind == "r":
                return "v%d" % (V_A + x)
            r = phys[v]
            return "v%d" % r if lo else "v[%d:%d]" % (r, r + 1)
        srcs = {}
        for k, s in enumerate(i.srcs):
            srcs["s%d" % k] = reg(s)
            if s[0] == "acc":
                srcs["s%dl" % k] = reg(s, lo=True)
        # free sources dying here before allocating the destination (no overlap issue: a
        # 64-bit op may write the pair it reads)
        for s in i.srcs:
            if s[0] == "acc" and last.get(s) == n and s in phys:
                free.append(phys.pop(s))
        if i.dst and i.dst[0] == "acc":
            if not free:
                raise SystemExit("accumulator pool exhausted")
            phys[i.dst] = free.pop(0)
        d = reg(i.dst) if i.dst else ""
        text.append(i.fmt.format(d=d, **srcs))
    return text


def outputs_safe(order):
    """Outputs r_j land in v[j]: a_j / the doubled limbs must be dead by then."""
    pos = {}
    for n, i in enumerate(order):
        for s in i.srcs:
            if s[0] == "a":
                pos[s[1]] = n
    for n, i in enumerate(order):
        if i.dst and i.dst[0] == "r":
            assert pos.get(i.dst[1], -1) < n, "output %d overwrites a live input" % i.dst[1]


def routine(name, square):
    ins, defs = build(square)
    order, cycles = schedule(ins, defs)
    outputs_safe(order)
    body = allocate(order, defs)
    head = ["s_mov_b32 s%d, 0x%x" % (S_P + j, P[j]) for j in range(NL)] + ["s_mov_b32 s%d, 0x%x" % (S_N0, N0)]
    lines = [".p2align 6", ".type %s,@function" % name, "%s:" % name] + head + body + \
        ["s_setpc_b64 s[%d:%d]" % (S_RET, S_RET + 1), ".size %s, .-%s" % (name, name)]
    nmad = sum(1 for i in ins if i.op == "mad")
    return lines, cycles, len(body), nmad


def wrappers():
    """Call sites: inline asm that pins the operands to the routines' registers and names the
    exact clobber set, so the compiler keeps everything else live across the call."""
    clob = ", ".join('"v%d"' % r for r in range(28, 62)) + ", " + ", ".join('"s%d"' % r for r in range(44, 64))
    call = ('"s_getpc_b64 s[62:63]\\n\\ts_add_u32 s62, s62, " SYM "@rel32@lo+4\\n\\t'
            's_addc_u32 s63, s63, " SYM "@rel32@hi+12\\n\\ts_swappc_b64 s[62:63], s[62:63]"')
    a_out = ", ".join('"+{v%d}"(r[%d])' % (i, i) for i in range(NL))
    b_in = ", ".join('"{v%d}"(b.v[%d])' % (14 + i, i) for i in range(NL))
    return [
        "",
        "#if defined(__HIPCC__) && (defined(BGV_ASM_MUL) || defined(BGV_ASM_EMIT))",
        "#define BGV_ASM_CALL(SYM) " + call,
        "#define BGV_ASM_CLOBBERS " + clob + ', "scc"',
        "// r = r b R^-1 (bgv_fpmul_x); operand limbs < 2^29, as fp_mul_l.  (The host pass of a HIP",
        "// unit compiles device bodies too: there the plain product stands in.)",
        "__device__ __forceinline__ void bgv_fpmul_asm(uint32_t r[14], const fp_t& b) {",
        "#if defined(__HIP_DEVICE_COMPILE__)",
        '  asm volatile(BGV_ASM_CALL("bgv_fpmul_x") : %s : %s : BGV_ASM_CLOBBERS);' % (a_out, b_in),
        "#else",
        "  fp_t a;",
        "  for (int i = 0; i < 14; ++i) a.v[i] = r[i];",
        "  const fp_t o = fp_mul_body(a, b);",
        "  for (int i = 0; i < 14; ++i) r[i] = o.v[i];",
        "#endif",
        "}",
        "// r = r^2 R^-1 (bgv_fpsqr_x)",
        "__device__ __forceinline__ void bgv_fpsqr_asm(uint32_t r[14]) {",
        "#if defined(__HIP_DEVICE_COMPILE__)",
        '  asm volatile(BGV_ASM_CALL("bgv_fpsqr_x") : %s : : BGV_ASM_CLOBBERS);' % a_out,
        "#else",
        "  fp_t a;",
        "  for (int i = 0; i < 14; ++i) a.v[i] = r[i];",
        "  const fp_t o = fp_sqr_body(a);",
        "  for (int i = 0; i < 14; ++i) r[i] = o.v[i];",
        "#endif",
        "}",
        "#endif",
    ]


def main():
    out = [
        "// GENERATED by tools/gen_fpmul_asm.py -- do not edit.",
        "// 28-bit-limb Montgomery product / square as gfx950 subroutines with a register contract of",
        "// their own: a = v[0:13], b = v[14:27] in, result in v[0:13]; clobbers v[28:61], s[44:63].",
        "// Bit-identical to fp_mul_body / fp_sqr_body (bls_field.h).  See the generator's docstring.",
        "#pragma once",
        "",
    ]
    asm = []
    stats = []
    for name, sq in (("bgv_fpmul_x", False), ("bgv_fpsqr_x", True)):
        lines, cycles, n, nmad = routine(name, sq)
        asm += lines
        stats.append("//   %s: %d VALU instructions (%d v_mad_u64_u32), modelled %d cycles at one wave per SIMD"
                     % (name, n, nmad, cycles))
    out += stats + [""]
    out.append("// Emitted only in units that use the routines (BGV_ASM_MUL, or BGV_ASM_EMIT for the")
    out.append("// microbenchmarks): the holder kernel's host symbol exists once per unit, so at most one")
    out.append("// unit of a library may define it.")
    out.append("#if defined(__HIPCC__) && (defined(BGV_ASM_MUL) || defined(BGV_ASM_EMIT))")
    out.append("// The routines live in the code of a kernel that is never launched (device compilation drops")
    out.append("// file-scope asm): one copy per kernel unit (no device linking), reached through the local")
    out.append("// labels by the call sites below.  The kernel ends before the first label.")
    out.append("__global__ void __launch_bounds__(64) bgv_fpmul_asm_holder() {")
    out.append("#if defined(__HIP_DEVICE_COMPILE__)")
    out.append("  asm volatile(")
    out.append('      "  s_endpgm\\n"')
    for ln in asm:
        out.append('      "  %s\\n"' % ln)
    out.append("  );")
    out.append("#endif")
    out.append("}")
    out.append("#endif")
    out += wrappers()
    open(OUT, "w").write("\n".join(out) + "\n")
    print("\n".join(stats))


if __name__ == "__main__":
    main()
