#!/bin/bash
# Fresh numbers for every config on one build (round start / round end).
# usage: bash scripts/baseline_box.sh <tag>
set -e
TAG=${1:-r03}
OUT=gpurun_out/base_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 200 python3 -u bench.py --config C2 --steps 2 --warmup 1 --e2e-steps 0 > $OUT/c2.json 2> $OUT/c2.err
timeout -k 10 200 python3 -u bench.py --config C4 --steps 2 --warmup 1 > $OUT/c4.json 2> $OUT/c4.err
timeout -k 10 200 python3 -u bench.py --config C1 --steps 3 --warmup 1 > $OUT/c1.json 2> $OUT/c1.err
