"""Summarise a scripts/profile_box.sh run: per-launch averages of the apply kernel's PMC counters
over the timed launches (the last `--launches` apply_kernel dispatches; the earlier ones are the
record-mode generation pass), with the gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md, HBM)."""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--launches", type=int, default=0, help="apply launches of the timed step (default: from kt.log)")
ap.add_argument("--kernel", default="apply_kernel")
ap.add_argument("--docs", type=int, default=100000)
ap.add_argument("--ops", type=int, default=1000)
ap.add_argument("--out", default=None)
a = ap.parse_args()

if not a.launches:  # the bench line of the kernel-trace run names the launches of one step
    for line in open(os.path.join(a.dir, "kt.log")):
        if line.startswith("{"):
            a.launches = json.loads(line)["roofline"]["launches_per_step"]
per = collections.Counter()
clock = []  # GHz per dispatch: GRBM_GUI_ACTIVE (8 XCDs' sum) / 8 / the dispatch's duration in ns
for f in sorted(glob.glob(os.path.join(a.dir, "*", "*_counter_collection.csv"))):
    d = collections.defaultdict(dict)
    dur = {}
    for r in csv.DictReader(open(f)):
        if a.kernel in r["Kernel_Name"]:
            d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            dur[int(r["Dispatch_Id"])] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    ids = sorted(d)[-a.launches:]
    for i in ids:
        if "GRBM_GUI_ACTIVE" in d[i] and dur.get(i, 0) > 0:
            clock.append(d[i]["GRBM_GUI_ACTIVE"] / 8.0 / dur[i])
    for i in ids:
        for k, v in d[i].items():
            per[k] += v / len(ids)
out = {"kernel": a.kernel, "docs": a.docs, "ops": a.ops, "launches_averaged": a.launches,
       "note_launches": "per-launch averages over the last `launches_averaged` apply dispatches (one timed step)"}
out["counters_per_launch"] = dict(per)
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    # FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads
    # (upper bound of the correction: our reads are 4-B-per-lane, so the raw value is a lower bound)
    fetch = per["FETCH_SIZE"] * 1024.0
    write = per["WRITE_SIZE"] * 1024.0
    out["hbm_read_bytes_per_launch_raw"] = fetch
    out["hbm_write_bytes_per_launch"] = write
    out["hbm_bytes_per_launch"] = 2.0 * fetch + write
    out["note"] = "hbm_bytes = 2*FETCH_SIZE (gfx950 correction) + WRITE_SIZE, KiB->bytes"
    out["hbm_bytes_per_step"] = out["hbm_bytes_per_launch"] * a.launches  # the averaged launches' total
if "SQ_LDS_BANK_CONFLICT" in per and "SQ_LDS_IDX_ACTIVE" in per:
    out["lds_bank_conflict_rate"] = per["SQ_LDS_BANK_CONFLICT"] / max(1.0, per["SQ_LDS_IDX_ACTIVE"])
if "SQ_WAVES" in per and "SQ_INSTS_VALU" in per:
    ops_per_launch = a.docs * a.ops / a.launches
    out["insts_per_op"] = {k[9:].lower(): per[k] / ops_per_launch for k in per if k.startswith("SQ_INSTS_")}
if clock:
    out["clock_ghz_measured"] = sum(clock) / len(clock)
    out["note_clock"] = "GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration, averaged over the same launches"
if "SQ_WAVE_CYCLES" in per:
    wc = per["SQ_WAVE_CYCLES"]
    out["wait_any_frac"] = per.get("SQ_WAIT_ANY", 0) / wc
    out["active_inst_frac"] = per.get("SQ_ACTIVE_INST_ANY", 0) / wc
s = json.dumps(out, indent=1)
print(s)
if a.out:
    open(a.out, "w").write(s + "\n")
