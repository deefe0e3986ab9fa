"""Print the fast traversal step of a trace kernel (`make asm` output) from its node-record
read: the instructions a common step issues.  Usage: python tools/step_isa.py FILE.s KERNEL [N]"""
import re
import sys

src = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 170
st = [i for i, l in enumerate(src) if re.match(r'^_Z\S*' + pat + r'\S*:', l)][0]
en = [i for i in range(st, len(src)) if src[i].startswith('.Lfunc_end')][0]
b = src[st:en]
k = [k for k, l in enumerate(b) if 'ds_read_b64' in l and 'offset:48' in l][0]
print('\n'.join(x for x in b[k - 12:k + n] if x.strip() and not x.strip().startswith(';')))
