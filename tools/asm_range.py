"""Instruction mix of lines [a, b) of a kernel in a hipcc -S listing
(line numbers relative to the kernel's label).
Usage: python tools/asm_range.py LISTING.s MANGLED_NAME a b"""
import collections
import sys

s = open(sys.argv[1]).read()
name, a, b = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
i = s.index(name + ':')
body = s[i:s.index('.Lfunc_end', i)].splitlines()[a:b]
c = collections.Counter(l.strip().split()[0] for l in body
                        if l.strip() and not l.strip().startswith((';', '.')))
mf = sum(v for k, v in c.items() if k.startswith('v_mfma'))
va = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
print("%d instructions, %d MFMA, %d other VALU" % (sum(c.values()), mf, va))
print("   " + ", ".join("%s %d" % kv for kv in c.most_common(30)))
