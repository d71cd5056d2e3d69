"""Count LDS / memory instruction kinds in one kernel of a `make asm` listing.

    python tools/asm_ds_count.py build/asm/NAME.s grad_kernelILi3ELi0E
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r'^(_Z\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M)
body = s[m.start():s.find('.Lfunc_end', m.start())]
c = collections.Counter(re.findall(r'^\s+((?:ds|global|buffer)_\w+)', body, re.M))
print(m.group(1)[:70])
for k, v in sorted(c.items()):
    print('  %-28s %d' % (k, v))
