# end-to-end knob sweep on C3 (bench.py's end_to_end leg): ops per launch of the pipelined run (MTR_PIPE_K)
set -e
mkdir -p gpurun_out/r06/sw
B="python -u bench.py --config C3 --steps 2 --no-cpu-baseline --e2e-steps 3"
for k in 0 144 192 48; do
  MTR_PIPE_K=$k timeout -k 10 300 $B > gpurun_out/r06/sw/pk$k.json 2>/dev/null
done
