"""Instruction histogram of one kernel in a hipcc -save-temps .s file.
    python tools/isa_census.py file.s substring
"""
import collections, sys
src = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
start = next(i for i, l in enumerate(src) if l.startswith('_Z') and key in l.split(':')[0])
ins = []
for l in src[start + 1:]:
    if 's_endpgm' in l:
        ins.append('s_endpgm'); break
    t = l.strip()
    if l.startswith('\t') and t and not t.startswith(('.', ';')):
        ins.append(t.split()[0])
c = collections.Counter(ins)
f64 = sum(v for k, v in c.items() if k.endswith('_f64'))
print(src[start].split(':')[0][:90])
print('total', len(ins), 'f64', f64, 'salu', sum(v for k, v in c.items() if k.startswith('s_')),
      'valu', sum(v for k, v in c.items() if k.startswith('v_')),
      'ds', sum(v for k, v in c.items() if k.startswith('ds_')))
print(c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30))
