#!/bin/bash
# PC sampling of the C3 apply kernel (line-table build libmtr_pcs.so:
# `python -m fluidframework_amd.build --variant pcs -gline-tables-only`), a 20k-document C3-shaped batch.
# host_trap first; stochastic only when host_trap exits with an ordinary error (no signal, no time limit).
# usage: bash scripts/pcsample_box.sh <tag> [docs]
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-r04}
DOCS=${2:-20000}
OUT=gpurun_out/pcs_$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1
echo "list rc=$?" >> $OUT/rc.txt
export MTR_LIB=libmtr_pcs.so
timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 -d $OUT/ht -o ht --output-format csv -- \
  python3 -u scripts/phase_profile.py --docs $DOCS --ops-per-launch 48 > $OUT/ht.log 2>&1
rc=$?
echo "host_trap rc=$rc" >> $OUT/rc.txt
if [ $rc -eq 0 ]; then exit 0; fi
if [ $rc -ne 1 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 65536 -d $OUT/st -o st --output-format csv -- \
  python3 -u scripts/phase_profile.py --docs $DOCS --ops-per-launch 48 > $OUT/st.log 2>&1
rc=$?
echo "stochastic rc=$rc" >> $OUT/rc.txt
exit $rc
