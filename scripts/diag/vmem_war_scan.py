"""Scan gfx950 device assembly (.s) for VMEM instructions whose address (or
store-data) VGPRs are overwritten by one of the next N instructions before
any wait -- the pattern of the one kernel instance that gave intermittent
wrong results (ftab_build_kernel<Geo<1,2,LAY_AC>>)."""
import re, sys, glob, collections

def regs(tok):
    m = re.match(r'[va]\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()

def scan(path, window):
    out = collections.Counter()
    kern = None
    lines = [l.strip() for l in open(path)]
    for i, l in enumerate(lines):
        if re.match(r'^_Z\w+:', l):
            kern = l.split(':')[0]
            continue
        m = re.match(r'(global|buffer|flat)_(load|store|atomic)\w*\s+(.*)', l)
        if not m or kern is None:
            continue
        ops = [o.strip() for o in m.group(3).split(',')]
        if m.group(2) == 'load':
            src = regs(ops[1]) if len(ops) > 1 else set()
        else:   # store / atomic: address and data
            src = set()
            for o in ops[:2]:
                src |= regs(o)
        if not src:
            continue
        j, n = i + 1, 0
        while j < len(lines) and n < window:
            t = lines[j]
            j += 1
            if not t or t.startswith(';') or t.startswith('.'):
                continue
            n += 1
            if t.startswith('s_waitcnt') or t.startswith('s_nop'):
                break
            mm = re.match(r'v_\w+(?:_e32|_e64)?\s+([va]\[?[\d:]+\]?)', t)
            if mm and regs(mm.group(1)) & src:
                out[kern] += 1
                break
    return out

window = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tot = collections.Counter()
for p in sorted(glob.glob(sys.argv[2] if len(sys.argv) > 2 else '/tmp/isa/*.s')):
    c = scan(p, window)
    for k, v in c.items():
        tot[k] += v
print(f"kernels with a VALU overwrite of VMEM source VGPRs within {window} instruction(s): {len(tot)}")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:60]:
    print(f"{v:4d}  {k[:150]}")
