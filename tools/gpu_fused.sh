#!/bin/bash
# fused-kernel bring-up: parity (fused vs unfused, bitwise) then a bench sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "${TESTS:-fused}" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_sweep.sh "$@"
