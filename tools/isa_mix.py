"""Static instruction mix of one kernel in a hipcc -S listing:
python tools/isa_mix.py <file.s> <substring of the mangled name> [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\S+):\s*;', s, re.M) + re.findall(r'^(_Z\S+):$', s, re.M)
sel = [n for n in names if all(p in n for p in sys.argv[2].split(','))]
for name in sel:
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    c = collections.Counter()
    for line in s[i:j].split('\n')[1:]:
        line = line.strip()
        if not line or line[0] in ';.' or line.endswith(':'):
            continue
        c[line.split()[0]] += 1
    print(name[:120], 'total', sum(c.values()))
    cls = collections.Counter()
    for op, n in c.items():
        k = ('v_f64' if op.endswith('_f64') and op.startswith('v_') else
             'v_other' if op.startswith('v_') else op.split('_')[0] + '_' + op.split('_')[1]
             if op.startswith(('ds_', 'global_', 'buffer_', 's_')) else op)
        cls[k] += n
    print(' classes:', dict(cls.most_common(12)))
    for op, n in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
        print(f'  {op:28s}{n}')
