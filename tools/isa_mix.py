"""Static instruction mix of kernels in a hipcc -S (gfx950) assembly file.
usage: python tools/isa_mix.py file.s mangled_name_substring..."""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    i = s.index(pat)
    i = s.rindex("\n", 0, i) + 1
    j = s.index(".Lfunc_end", i)
    body = [l.strip() for l in s[i:j].split("\n")]
    body = [l for l in body if l and not l.startswith((".", ";")) and not l.endswith(":")]
    c = Counter()
    for l in body:
        op = l.split()[0]
        c["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_")
          else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else op] += 1
    print(pat, len(body), dict(c))
    print("  ", Counter(l.split()[0] for l in body if l.startswith("v_")).most_common(16))
