#!/bin/bash
# quick parity subset + bench sweep: bash tools/gpu_quick_bench.sh "opts1" "opts2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "specialised or roundtrip or encode_512 or encode_batch" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_sweep.sh "$@"
