import re, sys
from collections import Counter
s = open(sys.argv[1]).read()
pat = sys.argv[2]
for m in re.finditer(r'^(\S*' + pat + r'\S*):\s*;', s, re.M):
    start = m.end()
    end = s.find('.Lfunc_end', start)
    body = s[start:end]
    ins = [l.strip().split()[0] for l in body.splitlines()
           if l.strip() and not l.strip().startswith(('.', ';', '_')) and not l.strip().endswith(':')]
    c = Counter(ins)
    print(m.group(1)[:90], 'total', len(ins))
    print('  ', ', '.join(f'{k} {v}' for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30)))
    meta = s[end:end + 3000]
    for key in ('NumVgprs', 'NumSgprs', 'ScratchSize', 'Occupancy'):
        mm = re.search(r'; ' + key + r': (\d+)', meta)
        if mm: print('  ', key, mm.group(1))
