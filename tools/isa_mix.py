"""Static instruction mix of kernels in a hipcc -S output: python isa_mix.py file.s pattern..."""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:]
for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S):
    name, body = m.group(1), m.group(2)
    if pats and not any(p in name for p in pats):
        continue
    c = collections.Counter()
    for line in body.split("\n"):
        t = line.strip()
        if not t or t.startswith((".", ";", "//")) or t.endswith(":"):
            continue
        x = t.split()[0]
        if x.startswith("v_mfma"): c["mfma"] += 1
        elif x.startswith(("v_readlane", "v_readfirstlane")): c["readlane"] += 1
        elif x.startswith("ds_bpermute"): c["bpermute"] += 1
        elif x.startswith("ds_"): c["ds"] += 1
        elif "_dpp" in t or "row_" in t: c["dpp"] += 1
        elif x.startswith("v_"): c["valu"] += 1
        elif x.startswith("s_waitcnt"): c["waitcnt"] += 1
        elif x.startswith("s_nop"): c["nop"] += 1
        elif x.startswith("s_"): c["salu"] += 1
        elif x.startswith(("global_", "buffer_", "scratch_")): c["vmem"] += 1
        else: c[x] += 1
    print(name, sum(c.values()), dict(c))
