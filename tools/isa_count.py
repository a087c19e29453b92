"""Instruction-class counts per kernel of a gfx950 assembly listing (hipcc --cuda-device-only -S).
    python tools/isa_count.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for f in re.split(r'\n(?=_Z\S+:)', s):
    m = re.match(r'(_Z\S+):', f)
    if not m or pat not in m.group(1):
        continue
    ins = [ln.split()[0] for ln in f.split('\n') if ln.startswith('\t') and not ln.strip().startswith(('.', ';'))]
    valu = [i for i in ins if i.startswith('v_')]
    mul = [i for i in valu if 'mul' in i or 'mad' in i]
    print(f"{m.group(1)[:90]:90s} valu {len(valu):6d} mul {len(mul):5d} "
          f"ds {sum(i.startswith('ds_') for i in ins):5d} vmem {sum(i.startswith(('global_', 'buffer_')) for i in ins):4d} "
          f"salu {sum(i.startswith('s_') for i in ins):5d}")
