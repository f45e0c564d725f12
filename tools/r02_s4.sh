#!/bin/bash
# Round-2 GPU session 4 (re-entry): confirm the restored tree — GPU test suite, default bench line.
set -o pipefail
O=gpurun_out/r02s4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > $O/b_default.json 2> $O/b_default.err || exit 1
cat $O/b_default.json
