#!/bin/bash
# FETCH_SIZE calibration of the decoders' per-lane stream reads (scripts/ubench/fetch_cal.hip)
export TMPDIR=/tmp
mkdir -p gpurun_out/cal
timeout -k 10 60 scripts/ubench/fetch_cal && \
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/cal/f -o run --output-format csv -- scripts/ubench/fetch_cal > gpurun_out/cal/f.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/cal/r -o run --output-format csv -- scripts/ubench/fetch_cal > gpurun_out/cal/r.log 2>&1
for f in $(find gpurun_out/cal -name "*counter_collection.csv"); do python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')): print(r['Kernel_Name'][:40], r['Counter_Name'], r['Counter_Value'])"; done
