set -e
mkdir -p gpurun_out/r05_base
timeout -k 10 300 python3 -u bench.py --config C3 --steps 5 --warmup 1 --e2e-steps 0 --no-cpu-baseline > gpurun_out/r05_base/C3.json 2> gpurun_out/r05_base/C3.err
