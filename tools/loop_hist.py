"""Instruction histogram of the hottest loop of a kernel in a hipcc -save-temps .s file."""
import collections
import re
import sys

path, kern = sys.argv[1], sys.argv[2]
s = open(path).read()
start = s.index(kern)
body = s[start:]
body = body[:body.index('.Lfunc_end')]
lines = [l.strip() for l in body.splitlines()]
lab = {}
for i, l in enumerate(lines):
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        lab[m.group(1)] = i
best = None
for i, l in enumerate(lines):
    m = re.match(r'^s_c?branch\w*\s+(\.LBB\d+_\d+)', l)
    if m and m.group(1) in lab and lab[m.group(1)] < i:
        span = i - lab[m.group(1)]
        if best is None or span > best[0]:
            best = (span, lab[m.group(1)], i)
_, a, b = best
loop = [l for l in lines[a:b + 1] if l and not l.startswith(('.', ';'))]
c = collections.Counter(l.split()[0] for l in loop)
half = sum(v for k, v in c.items() if k.startswith(('v_mad_u64', 'v_mul_lo', 'v_mul_hi')))
valu = sum(v for k, v in c.items() if k.startswith('v_'))
print(f"loop: {len(loop)} instr, VALU {valu} (half-rate {half}), est. VALU cycles/wave-iter {2*(valu-half)+4*half}")
for op, n in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
    print(f"  {op:30s}{n}")
