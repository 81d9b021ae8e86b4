"""Per-basic-block instruction mix of one kernel in a hipcc -save-temps .s file (dev tool).
usage: python tools/asm_stats.py file.s kernel_substring [min_mfma]"""
import re
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
min_mfma = int(sys.argv[3]) if len(sys.argv) > 3 else 1
s = open(src).read()
names = re.findall(r'^(_Z\S*):', s, re.M)
name = [n for n in names if pat in n][0]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
lines = s[i:j].split('\n')
blocks, cur, label = [], [], 'entry'
for ln in lines:
    m = re.match(r'^(\.LBB\S+|; %bb\.\d+):', ln.strip()) or re.match(r'^(\.LBB\S+):', ln)
    if m:
        blocks.append((label, cur)); cur = []; label = m.group(1)
        continue
    t = ln.strip()
    if t and not t.startswith(';') and not t.startswith('.'):
        cur.append(t.split()[0])
blocks.append((label, cur))
tot = Counter()
for lab, ins in blocks:
    c = Counter(ins)
    tot.update(c)
    mf = sum(v for k, v in c.items() if k.startswith('v_mfma'))
    if mf >= min_mfma:
        valu = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
        print(f"{lab:28s} n={len(ins):5d} mfma={mf:3d} valu={valu:4d} ds_read={sum(v for k,v in c.items() if k.startswith('ds_read')):3d} "
              f"scratch={sum(v for k,v in c.items() if k.startswith('scratch')):3d} waitcnt={c['s_waitcnt']:3d} nop={c['s_nop']:3d} "
              f"salu={sum(v for k,v in c.items() if k.startswith('s_') and k not in ('s_waitcnt','s_nop')):3d} vmem={sum(v for k,v in c.items() if k.startswith('global_')):3d}")
print('TOTAL scratch', sum(v for k, v in tot.items() if k.startswith('scratch')), 'mfma', sum(v for k, v in tot.items() if k.startswith('v_mfma')))
