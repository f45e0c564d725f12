#!/bin/bash
# one process per map-test case with a short limit: which case of tests/test_gpu_map_generator.py stalls
mkdir -p gpurun_out/r05bis
for L in pgtg_amd/libpgtg_hip.so ab/r04.so; do
  for k in $(seq 176 193); do
    PGTG_LIB=$PWD/$L timeout -k 5 40 python -u tests/test_gpu_map_generator.py $k >> gpurun_out/r05bis/cases.log 2>&1
    rc=$?
    echo "$L case $k rc=$rc" >> gpurun_out/r05bis/cases.log
    [ $rc -eq 0 ] || { cat gpurun_out/r05bis/cases.log; exit 1; }
  done
done
cat gpurun_out/r05bis/cases.log
