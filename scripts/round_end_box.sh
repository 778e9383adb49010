#!/bin/bash
# Round-end measurements on one build: GPU suite, smoke, every config's bench line (C5 with its CPU
# baseline), then the C3 kernel-trace + PMC passes (scripts/profile_box.sh).  Each step has its own
# time limit; the first failure ends the script.
# usage: bash scripts/round_end_box.sh <tag>
set -e
TAG=${1:-r03_end}
OUT=gpurun_out/end_$TAG
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash scripts/baseline_box.sh $TAG
# C2 / C4 may not drop more than 2 % below the previous round's end lines (REF: profiles/<round>_bench_c*_end.json)
REF=${REF:-r03}
python3 scripts/regress_check.py --tol 0.02 gpurun_out/base_$TAG/c2.json:profiles/${REF}_bench_c2_end.json \
  gpurun_out/base_$TAG/c4.json:profiles/${REF}_bench_c4_end.json gpurun_out/base_$TAG/c3.json:profiles/${REF}_bench_c3_end.json \
  > $OUT/regress.txt 2>&1
timeout -k 10 600 python3 -u bench.py --config C5 --steps 1 --warmup 0 > gpurun_out/base_$TAG/c5.json 2> gpurun_out/base_$TAG/c5.err
bash scripts/profile_box.sh $TAG --steps 1 --warmup 0 --no-cpu-baseline > $OUT/profile.log 2>&1
echo done > $OUT/done
