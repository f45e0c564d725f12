#!/bin/bash
# Round-2 GPU session 2b: velocity sweep + exhaustive parity, then the whole GPU suite.
set -o pipefail
O=gpurun_out/r02s2
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_velocity.py tests/test_gpu_exhaustive.py > $O/new_tests2.log 2>&1
echo "new tests rc=$?"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/new_tests2.log | tail -40
