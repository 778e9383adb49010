set -e
TAG=r03_end
OUT=gpurun_out/end_$TAG
mkdir -p $OUT gpurun_out/base_$TAG
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash scripts/baseline_box.sh $TAG
timeout -k 10 600 python3 -u bench.py --config C5 --steps 1 --warmup 0 > gpurun_out/base_$TAG/c5.json 2> gpurun_out/base_$TAG/c5.err
