"""Instruction counts per basic block of the fast traversal loop in the hot trace kernel's ISA
(`make asm` output): how DESIGN.md §3.2 items 19-20 were sized before any GPU run.
Usage: python tools/loop_isa.py gpu-ray-tracer_amd/build/rt_kernels.s [kernel-substring]"""
import re, sys, collections
src = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2] if len(sys.argv) > 2 else 'trace_kernelILi2ELb1ELi180E'
st = [i for i, l in enumerate(src) if re.match(r'^_Z\S*' + pat + r'\S*:', l)][0]
en = [i for i in range(st, len(src)) if src[i].startswith('.Lfunc_end')][0]
body = src[st:en]
# the pair step: a block with ds_read_b64 .. offset:48 followed by ds_read_b128
hdr, depth = None, None
for i, l in enumerate(body):
    if 'ds_read_b64' in l and 'offset:48' in l and 'ds_read_b128' in body[i + 1]:
        for j in range(i, 0, -1):
            m = re.search(r'Header=(BB\d+_\d+) Depth=(\d+)', body[j])
            if m: hdr = m.group(1); depth = m.group(2); break
        break
print('loop header', hdr, 'depth', depth)
blocks = collections.OrderedDict(); cur = None
for l in body:
    m = re.match(r'^\.L(BB\d+_\d+):(.*)', l)
    if m:
        cur = m.group(1) if ('Header=' + hdr in m.group(2) or m.group(1) == hdr) else None
        if cur: blocks[cur] = collections.Counter()
        continue
    if cur and l.startswith('\t') and not l.strip().startswith(('.', ';')):
        op = l.split()[0]
        if op.startswith('v_'): k = 'valu'
        elif op.startswith(('s_cbranch', 's_branch')): k = 'branch'
        elif op.startswith('s_waitcnt') or op.startswith('s_nop'): k = 'wait/nop'
        elif op.startswith(('s_load', 's_buffer')): k = 'smem'
        elif op.startswith('s_'): k = 'salu'
        elif op.startswith('ds_'): k = 'lds'
        else: k = 'other'
        blocks[cur][k] += 1
tot = collections.Counter()
for b, c in blocks.items():
    tot.update(c)
    print('%-10s %s' % (b, dict(c)))
print('TOTAL blocks', len(blocks), dict(tot))
