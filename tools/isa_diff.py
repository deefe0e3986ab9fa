"""Compare the per-kernel instruction streams of two `make asm` listings (labels and
comments normalised): used to show that a source change leaves the shipped kernels'
code unchanged (e.g. removing dead A/B arms)."""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r'^(_Z\S+):\s', line)
        if m and not line.startswith('\t'):
            cur, body = m.group(1), []
            continue
        if cur and line.startswith('.Lfunc_end'):
            out[cur] = body
            cur = None
            continue
        if cur:
            t = line.split(';')[0].strip()
            if not t or t.startswith('.'):
                continue
            t = re.sub(r'\.LBB\d+_\d+', 'L', t)
            out.setdefault(cur, None)
            body.append(t)
    return out


def meta(path):
    txt = open(path).read()
    res = {}
    for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)(?=\n  - \.|\Z)', txt, re.S):
        blk = m.group(2)
        g = {k: re.search(r'\.%s:\s+(\d+)' % k, blk) for k in ('sgpr_spill_count', 'vgpr_spill_count', 'vgpr_count', 'private_segment_fixed_size')}
        res[m.group(1)] = {k: int(v.group(1)) for k, v in g.items() if v}
    return res


if __name__ == '__main__':
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    ma, mb = meta(sys.argv[1]), meta(sys.argv[2])
    pat = sys.argv[3] if len(sys.argv) > 3 else ''
    for k in sorted(set(a) | set(b)):
        if pat not in k:
            continue
        if k not in a or k not in b:
            print('only in %s: %s' % ('old' if k in a else 'new', k))
            continue
        same = a[k] == b[k]
        print('%-4s %6d -> %6d instr  %s  %s -> %s' % ('same' if same else 'DIFF', len(a[k]), len(b[k]), k[:90],
                                                      ma.get(k, {}), mb.get(k, {})))
