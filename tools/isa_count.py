"""Static instruction mix of the kernels in a hipcc device assembly file.

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -o k.s file.hip
    python tools/isa_count.py k.s [substring-of-kernel-name]
"""
import re
import sys
from collections import Counter


def kernels(path):
    s = open(path).read()
    for m in re.finditer(r'^(_Z\w+):\s*;', s, re.M):
        name = m.group(1)
        end = s.find('.Lfunc_end', m.end())
        yield name, s[m.end():end]


def mix(body):
    c = Counter()
    for raw in body.split('\n'):
        l = raw.strip()
        if not l or l.startswith(('.', ';', '//')) or l.endswith(':'):
            continue
        op = l.split()[0]
        if op.startswith('s_waitcnt'):
            c['s_waitcnt'] += 1
        elif op.startswith(('s_cbranch', 's_branch')):
            c['branch'] += 1
        elif op.startswith('s_'):
            c['salu'] += 1
            c['salu:' + op] += 1
        elif op.startswith('v_mfma'):
            c['mfma'] += 1
        elif op.startswith('v_pk_'):
            c['valu'] += 1
            c['valu_pk'] += 1
        elif op.startswith('v_'):
            c['valu'] += 1
        elif op.startswith('ds_'):
            c['lds'] += 1
        elif op.startswith(('buffer', 'global', 'flat')):
            c['vmem'] += 1
        else:
            c['other:' + op] += 1
    return c


if __name__ == '__main__':
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ''
    for name, body in kernels(path):
        if sub in name:
            c = mix(body)
            top = ', '.join(f'{k}={v}' for k, v in c.most_common(14) if not k.startswith('salu:'))
            sal = ', '.join(f'{k[5:]}={v}' for k, v in c.most_common() if k.startswith('salu:'))[:300]
            print(f'{name}\n  {top}\n  salu: {sal}')
