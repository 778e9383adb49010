# end-to-end A/B on C3 (bench.py's end_to_end leg): ramped first parts (default) against equal parts
set -e
mkdir -p gpurun_out/r06/sw
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py -k pipelined > gpurun_out/r06/sw/tests.log 2>&1
B="python -u bench.py --config C3 --steps 2 --no-cpu-baseline --e2e-steps 3"
for r in 1 0 1 0; do
  MTR_PIPE_RAMP=$r timeout -k 10 300 $B > gpurun_out/r06/sw/ramp$r.$RANDOM.json 2>/dev/null
done
