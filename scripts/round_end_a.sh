#!/bin/bash
# Round-end measurements, part A (one build): the GPU suite, smoke, every config's bench line with its CPU baseline
# (C3 5 steps), the regression guard against the previous round's end lines, C5.  A failure ends the script.
# usage: bash scripts/round_end_a.sh <tag>     (REF=<previous round> for the guard, default r03)
set -e
TAG=${1:-r05_end}
OUT=gpurun_out/end_$TAG
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash scripts/baseline_box.sh $TAG
REF=${REF:-r04}
python3 scripts/regress_check.py --tol 0.02 gpurun_out/base_$TAG/c2.json:profiles/${REF}_bench_c2_end.json \
  gpurun_out/base_$TAG/c4.json:profiles/${REF}_bench_c4_end.json gpurun_out/base_$TAG/c3.json:profiles/${REF}_bench_c3_end.json \
  > $OUT/regress.txt 2>&1
timeout -k 10 600 python3 -u bench.py --config C5 --steps 1 --warmup 0 > gpurun_out/base_$TAG/c5.json 2> gpurun_out/base_$TAG/c5.err
echo done > $OUT/done
