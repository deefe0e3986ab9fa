"""SGPR spill census of a trace kernel (`make asm` output): ISA metadata (SGPR / VGPR spills,
scratch) and the v_readlane / v_writelane spill restores and saves by loop, so that the cost of
the spills is placed: per group (the persistent group loop), per state-machine iteration (one
per wave query), or per traversal step.  The traversal stack's own lane moves (M0 / SGPR-indexed)
are left out.  Usage: python tools/spill_census.py gpu-ray-tracer_amd/build/rt_kernels.s [kernel-substring]"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else 'trace_kernelILi0ELb1ELi180E'
for b in src.split('  - .agpr_count'):
    n = re.search(r'\.name:\s+(\S+)', b)
    if n and pat in n.group(1):
        print(n.group(1))
        for k in ('sgpr_count', 'sgpr_spill_count', 'vgpr_count', 'vgpr_spill_count', 'private_segment_fixed_size'):
            print('  %-28s %s' % (k, re.search(r'\.%s:\s+(\d+)' % k, b).group(1)))
lines = src.split('\n')
st = [i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + pat + r'\S*:', l)][0]
en = [i for i in range(st, len(lines)) if lines[i].startswith('.Lfunc_end')][0]
depth, per = 0, collections.Counter()
n_inst = 0
for l in lines[st:en]:
    m = re.match(r'^\.L(BB\d+_\d+):(.*)', l)
    if m:
        d = re.search(r'Depth=(\d+)', m.group(2))
        depth = int(d.group(1)) if d else 0
        continue
    s = l.strip()
    if not s or s.startswith(('.', ';')):
        continue
    n_inst += 1
    op = s.split()[0]
    if op == 'v_readlane_b32' and not re.search(r', s\d+$', s):          # not an SGPR-indexed (stack) read
        per[(depth, 'restore')] += 1
    if op == 'v_writelane_b32' and 'm0' not in s:
        per[(depth, 'save')] += 1
print('instructions', n_inst)
names = {0: 'kernel prologue/epilogue', 1: 'group loop', 2: 'state machine (per wave query)',
         3: 'traversal step', 4: 'leaf / triangle loops', 5: 'inner loops'}
for (d, k), v in sorted(per.items()):
    print('  depth %d %-32s %-8s %d (static)' % (d, names.get(d, 'deeper loops'), k, v))
