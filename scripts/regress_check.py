"""Round-end regression guard: fail when a config's bench line drops more than `--tol` below its reference
line (the previous round's end, or this round's start).  usage:
python scripts/regress_check.py --tol 0.02 <new.json>:<reference.json> [...]"""
import argparse
import json
import sys


def value(path):
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)["value"], json.loads(line)["config"].get("workload", "")
    raise SystemExit(f"{path}: no bench line")


ap = argparse.ArgumentParser()
ap.add_argument("--tol", type=float, default=0.02)
ap.add_argument("pairs", nargs="+")
a = ap.parse_args()
bad = 0
for pair in a.pairs:
    new, ref = pair.split(":")
    v, w = value(new)
    r, _ = value(ref)
    ok = v >= (1.0 - a.tol) * r
    bad += not ok
    print(f"{'ok  ' if ok else 'FAIL'} {w[:40]:40s} {v / 1e6:9.2f} M vs {r / 1e6:9.2f} M ({(v / r - 1) * 100:+.1f} %)")
sys.exit(1 if bad else 0)
