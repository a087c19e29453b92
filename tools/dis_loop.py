"""Instruction mix of the largest backward-branch loop in an llvm-objdump listing of one kernel
(tools/dis_loop.py k.dis): VALU / multiplies / LDS / VMEM / barriers per iteration."""
import collections, re, sys

lines = [l for l in open(sys.argv[1]) if re.match(r'^\s+[sv]_|^\s+(ds|global|buffer|scratch|flat)_', l)]
addr = []
for l in lines:
    m = re.search(r'// ([0-9A-F]{12}):', l)
    addr.append(int(m.group(1), 16) if m else None)
best = None
for i, l in enumerate(lines):
    m = re.match(r'^\s+s_c?branch\w*\s+(\d+)', l)
    if m and addr[i] is not None:
        off = int(m.group(1))
        if off >= 32768:  # backward (simm16)
            tgt = addr[i] + 4 + (off - 65536) * 4
            j = addr.index(tgt) if tgt in addr else None
            # the loop with the most barriers, then the longest (the accumulator loop, not a division loop)
            key = lambda jj, ii: (sum('s_barrier' in x for x in lines[jj:ii + 1]), ii - jj)
            if j is not None and (best is None or key(j, i) > key(*best)):
                best = (j, i)
a, b = best
c = collections.Counter(l.split()[0] for l in lines[a:b + 1])
mul = sum(v for k, v in c.items() if k.startswith(('v_mad_u64', 'v_mad_i64', 'v_mul_lo', 'v_mul_hi')))
valu = sum(v for k, v in c.items() if k.startswith('v_'))
lds = sum(v for k, v in c.items() if k.startswith('ds_'))
vmem = sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_', 'scratch_', 'flat_')))
print(f"loop: {b - a + 1} instr, VALU {valu} (multiplies {mul}), LDS {lds}, VMEM {vmem}, "
      f"barrier {c['s_barrier']}, waitcnt {c['s_waitcnt']}, nop {c['s_nop']}")
for op, n in c.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 12):
    print(f"  {op:28s}{n}")
