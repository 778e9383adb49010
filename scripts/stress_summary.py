"""Summarise scripts/r05_stress.sh: per run, its shape, ops/s and the bit-exact sample."""
import glob
import json
import os
import sys

rows = []
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        rows.append({"run": os.path.basename(f)[:-5], "error": "no bench line"})
        continue
    d = json.loads(lines[-1])
    c = d["config"]
    rows.append({"run": os.path.basename(f)[:-5], "docs": c.get("docs_per_gpu", c.get("docs")), "ops": c.get("ops_per_doc"),
                 "writers": c.get("writers"), "max_lag": c.get("max_lag"), "mops": round(d["value"] / 1e6, 2),
                 **d["bit_exact_sample"]})
ok = all(r.get("equal") == r.get("checked_docs") and r.get("checked_docs") for r in rows)
print(json.dumps({"runs": rows, "all_bit_exact": ok}, indent=1))
