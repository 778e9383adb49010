#!/bin/bash
# Bench several engine builds (libmtr_<name>.so, python -m fluidframework_amd.build --variant ...) in one
# GPU session: one short C3 bench per library, each under its own time limit.
# usage: bash scripts/variants.sh "<bench args>" lib1.so lib2.so ...
ARGS=$1; shift
mkdir -p gpurun_out/variants
for lib in "$@"; do
    MTR_LIB=$lib timeout -k 10 240 python3 -u bench.py $ARGS --no-cpu-baseline --e2e-steps 0 \
        > gpurun_out/variants/$lib.log 2>&1 || { echo "$lib failed rc=$?"; tail -3 gpurun_out/variants/$lib.log; exit 1; }
    python3 - "$lib" <<'PY'
import json, sys
lib = sys.argv[1]
line = [l for l in open(f"gpurun_out/variants/{lib}.log") if l.startswith("{")][-1]
r = json.loads(line)
print(f"{lib:28s} {r['value']/1e6:8.1f} M ops/s  apply {r['detail']['apply_ms_per_step']:7.1f} ms  "
      f"avg launch {r['roofline']['avg_launch_ms']:.3f} ms  digest {r['detail']['digest']}")
PY
done
