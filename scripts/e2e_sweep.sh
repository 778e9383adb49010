# end-to-end A/B on C3 (bench.py's end_to_end leg): class width of the pipelined run (MTR_CLASS_LEAVES)
set -e
mkdir -p gpurun_out/r06/sw3
B="python -u bench.py --config C3 --steps 2 --no-cpu-baseline --e2e-steps 3"
for c in 0 128 0 128; do
  if [ $c = 0 ]; then timeout -k 10 300 $B > gpurun_out/r06/sw3/c$c.$RANDOM.json 2>/dev/null;
  else MTR_CLASS_LEAVES=$c timeout -k 10 300 $B > gpurun_out/r06/sw3/c$c.$RANDOM.json 2>/dev/null; fi
done
