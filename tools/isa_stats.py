"""Per-function register / scratch / instruction statistics of a gfx950 assembly file
(hipcc --cuda-device-only -S): the tool behind the spill and code-size figures in DESIGN.md.

    python tools/isa_stats.py file.s [name-substring ...]
"""
import collections
import re
import subprocess
import sys


def stats(path):
    funcs, cur = {}, None
    for ln in open(path):
        m = re.match(r'^([_a-zA-Z][_a-zA-Z0-9.]*):', ln)
        if m and not ln.startswith('.L'):
            cur = m.group(1)
            funcs[cur] = collections.Counter()
            continue
        if cur is None:
            continue
        m = re.match(r'^; (NumVgprs|NumAgprs|ScratchSize|codeLenInByte)[:=] *=? *(\d+)', ln)
        if m:
            funcs[cur][m.group(1)] = int(m.group(2))
            continue
        t = ln.split()
        if not t or t[0].startswith(('.', ';')):
            continue
        op = t[0]
        c = funcs[cur]
        if op.startswith(('scratch_', 'buffer_')):
            c['scratch'] += 1
        elif op.startswith('v_accvgpr'):
            c['accv'] += 1
        elif op == 's_swappc_b64':
            c['call'] += 1
        elif op.startswith('v_mad_u64_u32'):
            c['mad'] += 1
            c['valu'] += 1
        elif op.startswith('v_'):
            c['valu'] += 1
    return funcs


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    for f, c in stats(path).items():
        if c['valu'] < 50 and not c.get('ScratchSize'):
            continue
        dn = subprocess.run(['c++filt', f], capture_output=True, text=True).stdout.strip()
        if pats and not any(p in dn for p in pats):
            continue
        print("%-60s v=%3d a=%3d scratch=%5d | valu=%6d mad=%6d scr_ops=%5d accv=%5d calls=%4d" % (
            dn[:60], c['NumVgprs'], c['NumAgprs'], c['ScratchSize'], c['valu'], c['mad'], c['scratch'], c['accv'],
            c['call']))


if __name__ == '__main__':
    main()
