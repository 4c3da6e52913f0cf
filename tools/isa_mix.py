"""Static instruction mix of device kernels (from hipcc -S output).

python tools/isa_mix.py /tmp/gh.s <mangled-name-substring> [...]
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:]
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):", s, re.M)]
for i, (pos, name) in enumerate(starts):
    if not all(p in name for p in pats):
        continue
    end = starts[i + 1][0] if i + 1 < len(starts) else len(s)
    body = s[pos:end]
    body = body.split("s_endpgm")[0]
    ops = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ops)
    cat = collections.Counter()
    for op, n in c.items():
        if op.startswith("v_") and "f64" in op:
            cat["valu_f64"] += n
        elif op.startswith("v_"):
            cat["valu_other"] += n
        elif op.startswith("s_"):
            cat["salu"] += n
        elif op.startswith(("global", "buffer", "flat")):
            cat["vmem"] += n
        elif op.startswith("ds_"):
            cat["lds"] += n
        else:
            cat[op] += n
    print(name, len(ops), dict(cat))
    for op, n in c.most_common(40):
        print(f"   {op:30s}{n}")
