"""Scan hipcc device assembly for a VMEM store of more than 8 bytes whose data VGPRs are
overwritten by one of the next two instructions (no wait state between): on gfx950 the store
can read its data after that write (seen as corrupt output in some lanes), so such a store
needs an `s_nop 1` after it.  Usage: python tools/store_hazard_scan.py file.s [...]"""
import re
import sys


def vregs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def scan(path):
    s = open(path).read()
    found = []
    for m in re.finditer(r'^(_Z\w+):\s*;', s, re.M):
        body = [l.strip() for l in s[m.end():s.find('.Lfunc_end', m.end())].split('\n')]
        body = [l for l in body if l and not l.startswith(('.', ';', '//')) and not l.endswith(':')]
        for i, l in enumerate(body):
            op = l.split()[0]
            if not re.match(r'(buffer|global|flat)_store_(dwordx[34]|b96|b128)', op):
                continue
            ops = [o.strip() for o in l[len(op):].split(',')]
            data = vregs(ops[1] if op.startswith(('global', 'flat')) else ops[0])
            for nxt in body[i + 1:i + 3]:
                if nxt.startswith('s_nop'):
                    break
                mm = re.match(r'(v_\w+)\s+(v\[\d+:\d+\]|v\d+)', nxt)
                if mm and not mm.group(1).startswith('v_cmp') and vregs(mm.group(2)) & data:
                    found.append((m.group(1), l, nxt))
                    break
    return found


if __name__ == '__main__':
    total = 0
    for p in sys.argv[1:]:
        for fn, st, nxt in scan(p):
            total += 1
            print(f'{p}: {fn[:60]}: {st}  ->  {nxt}')
    print('hazards', total)
