"""Scratch (spill) load/store sites of a kernel in `make asm` output, with their loop depth.
Usage: python tools/scratch_sites.py gpu-ray-tracer_amd/build/rt_kernels.s KERNEL-SUBSTRING"""
import re
import sys

src = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
st = [i for i, l in enumerate(src) if re.match(r'^_Z\S*' + pat + r'\S*:', l)][0]
en = [i for i in range(st, len(src)) if src[i].startswith('.Lfunc_end')][0]
depth, blk = 0, '-'
for i in range(st, en):
    l = src[i]
    m = re.match(r'^\.L(BB\d+_\d+):(.*)', l)
    if m:
        d = re.search(r'Depth=(\d+)', m.group(2))
        depth, blk = (int(d.group(1)) if d else 0), m.group(1)
        continue
    if 'scratch_' in l:
        print(depth, blk, l.strip())
