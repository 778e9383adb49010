"""Side by side: two phase_profile.py outputs (cycles per op per phase, and the per-op counts)."""
import json
import sys

a, b = (json.load(open(p)) for p in sys.argv[1:3])
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 300
print(f"apply_ms {a['apply_ms']:.1f} vs {b['apply_ms']:.1f}")
for k in a["phases"]:
    x = a["phases"][k]["cycles_per_op"]
    y = b["phases"].get(k, {}).get("cycles_per_op", 0)
    if x > thr or y > thr:
        print(f"{k:14s} {x:10.0f} {a['phases'][k]['frac_of_op']:6.3f}   {y:10.0f}")
print({k: round(v, 3) for k, v in a["per_op_counts"].items() if v})
