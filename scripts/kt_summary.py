"""Summarise a rocprofv3 --kernel-trace run of bench.py (scripts/profile_box.sh): the apply kernel's
dispatches of the timed step (the last `launches_per_step` ones; the earlier ones belong to the
untimed record-mode generation), their average duration (to compare with bench.py's
roofline.avg_launch_ms) and the step's span."""
import csv
import json
import os
import sys

d = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None
bench = None
for line in open(os.path.join(d, "kt.log")):
    if line.startswith("{"):
        bench = json.loads(line)
n = bench["roofline"]["launches_per_step"]
rows = list(csv.DictReader(open(os.path.join(d, "kt", "kt_kernel_trace.csv"))))
# the timed kernel: apply_kernel (SharedString configs) or apply_pair_kernel (C4 matrices)
kern = "apply_pair_kernel" if "apply_pair_kernel" in bench["roofline"].get("kernel", "") else "apply_kernel"
ak = [r for r in rows if kern in r["Kernel_Name"]][-n:]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ak]
t0 = min(int(r["Start_Timestamp"]) for r in ak)
t1 = max(int(r["End_Timestamp"]) for r in ak)
by = {}
for r, x in zip(ak, dur):
    k = r["Kernel_Name"]
    c, s = by.get(k, (0, 0.0))
    by[k] = (c + 1, s + x)
res = {
    "source": "rocprofv3 --kernel-trace --stats -- python3 bench.py " + " ".join(sys.argv[3:]),
    "timed_step_apply_launches": n,
    "avg_launch_ms_rocprof": sum(dur) / n,
    "avg_launch_ms_bench_hip_events": bench["roofline"]["per_launch"]["avg_launch_ms"],
    "apply_span_ms_rocprof": (t1 - t0) / 1e6,
    "apply_wall_ms_bench": bench["roofline"].get("apply_wall_ms_per_step"),
    "bench_value_under_profiler": bench["value"],
    "per_instantiation": {k: {"calls": c, "avg_ms": s / c} for k, (c, s) in sorted(by.items())},
}
s = json.dumps(res, indent=1)
print(s)
if out:
    open(out, "w").write(s + "\n")
