"""Static instruction mix of one kernel in a hipcc -S assembly file (tools/diag, CPU only).
usage: python tools/diag/isa_mix.py file.s <mangled-name-substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
starts = [m for m in re.finditer(r"^(_Z\S+):", s, re.M) if sys.argv[2] in m.group(1)]
if not starts:
    sys.exit("no such kernel")
a = starts[0].end()
e = s.find("s_endpgm", a)
e = s.find(".Lfunc_end", e)
body = s[a:e]
ins = [l.split()[0] for l in body.splitlines() if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
cls = collections.Counter()
for i in ins:
    cls["v_" if i.startswith("v_") else i.split("_")[0] + "_"] += 1
print(starts[0].group(1)[:90], "instructions:", len(ins))
print(cls.most_common(10))
print(collections.Counter(i for i in ins if i.startswith("v_")).most_common(30))
