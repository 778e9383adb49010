set -e
OUT=gpurun_out/end_c5
mkdir -p $OUT
timeout -k 10 600 python3 -u bench.py --config C5 --steps 1 --warmup 0 > $OUT/c5.json 2> $OUT/c5.err
bash scripts/profile_box.sh r03_c5end --config C5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/profile.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/prof_r03_c5end --kernel "apply_kernel<true, -1" --launches 43 --docs 1000 --ops 20000 --out $OUT/traffic_r03_c5.json > /dev/null
rm -f gpurun_out/prof_r03_c5end/kt/kt_kernel_trace.csv gpurun_out/prof_r03_c5end/*/*_counter_collection.csv
MTR_LIB=libmtr_prof.so timeout -k 10 400 python3 -u scripts/phase_profile.py --grow 200000 --ops 20000 --writers 64 --max-lag 4096 --docs 64 --ops-per-launch 512 > $OUT/phase_c5.json 2> $OUT/phase_c5.err
