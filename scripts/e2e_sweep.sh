set -e
mkdir -p gpurun_out/r06/sw
B="python -u bench.py --config C3 --steps 2 --no-cpu-baseline --e2e-steps 2"
timeout -k 10 300 $B > gpurun_out/r06/sw/base.json 2>/dev/null
timeout -k 10 300 $B --ops-per-launch 96 > gpurun_out/r06/sw/k96.json 2>/dev/null
MTR_SLACK=24 timeout -k 10 300 $B > gpurun_out/r06/sw/s24.json 2>/dev/null
MTR_SLACK=24 timeout -k 10 300 $B --ops-per-launch 96 > gpurun_out/r06/sw/k96s24.json 2>/dev/null
