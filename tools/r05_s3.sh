#!/bin/bash
# round 5 session 3: SQ instruction counters of k_envq (configs[4]), r04 vs new
set -o pipefail
O=gpurun_out/r05s3; mkdir -p $O
PGTG_LIB=$PWD/ab/r04.so timeout -k 10 300 bash tools/sq_passes.sh r04 cfg5 k_envq > $O/sq_r04.txt 2>&1 || { tail $O/sq_r04.txt; exit 1; }
timeout -k 10 300 bash tools/sq_passes.sh new cfg5 k_envq > $O/sq_new.txt 2>&1 || { tail $O/sq_new.txt; exit 1; }
tail -2 $O/sq_r04.txt $O/sq_new.txt
