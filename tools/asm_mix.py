"""Instruction mix of a kernel's MFMA loop in a hipcc -S listing (the loop,
among those LLVM marks 'Loop Header', that holds the most v_mfma).
Usage: python tools/asm_mix.py LISTING.s MANGLED_NAME [MANGLED_NAME ...]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for name in sys.argv[2:]:
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    body = s[i:j].splitlines()
    best = None
    for h, l in enumerate(body):
        m = re.match(r'(\.LBB\d+_\d+):.*Loop Header', l)
        if not m:
            continue
        lab = m.group(1)
        br = [k for k, x in enumerate(body) if 'branch' in x and re.search(re.escape(lab) + r'\b', x)]
        a, b = min([h] + br), max([h] + br)
        nm = sum('v_mfma' in x for x in body[a:b + 1])
        if best is None or nm > best[0]:
            best = (nm, a, b)
    _, a, b = best
    c = collections.Counter()
    for l in body[a:b + 1]:
        l = l.strip()
        if l and not l.startswith((';', '.')):
            c[l.split()[0]] += 1
    mf = sum(v for k, v in c.items() if k.startswith('v_mfma'))
    va = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
    print("%s: loop lines %d-%d, %d instructions, %d MFMA, %d other VALU" %
          (name, a, b, sum(c.values()), mf, va))
    print("   " + ", ".join("%s %d" % kv for kv in c.most_common(30)))
