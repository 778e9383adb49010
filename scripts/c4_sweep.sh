#!/bin/bash
# C4 launch-parameter sweep (no CPU leg): default, HBM-resident pairs, ops per launch
set -e
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/c4_$name.log 2>&1; }
run base python bench.py --config C4 --steps 2 --no-cpu-baseline
MTR_LDS_LIMIT=0 run global python bench.py --config C4 --steps 2 --no-cpu-baseline
run k96 python bench.py --config C4 --steps 2 --no-cpu-baseline --ops-per-launch 96
run k16 python bench.py --config C4 --steps 2 --no-cpu-baseline --ops-per-launch 16
