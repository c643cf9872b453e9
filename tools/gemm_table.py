"""Tabulate tools/gemm_bench.py logs side by side: python tools/gemm_table.py a.log [b.log ...]"""
import json
import sys
from collections import defaultdict

for f in sys.argv[1:]:
    d = defaultdict(dict)
    for l in open(f):
        if l.startswith('{"shape"') and '"cfg"' in l:
            r = json.loads(l)
            d[r["shape"]][r["cfg"]] = r["us"]
    cfgs = []
    for v in d.values():
        cfgs += [c for c in v if c not in cfgs]
    print(f)
    print("cfg      " + " ".join(f"{s[:10]:>10}" for s in d))
    for c in cfgs:
        print(f"{c:8s} " + " ".join(f"{d[s].get(c, float('nan')):10.1f}" for s in d))
