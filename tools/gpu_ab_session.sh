#!/bin/bash
# One GPU session for a candidate build: the GPU test suite, then an interleaved A/B of the in-tree
# library against another build on the given workloads.  Usage: bash tools/gpu_ab_session.sh <other.so> <workloads...>
O=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
tail -2 gpurun_out/ab_tests.log
grep -q " passed" gpurun_out/ab_tests.log && ! grep -q "failed\|error" gpurun_out/ab_tests.log || exit 1
bash tools/ab.sh "$O" "$@"
