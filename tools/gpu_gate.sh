#!/bin/bash
# VERDICT r5 item 2's gate on one GPU: the new bench-scale tests (verbose), then
# tools/gate_probe.py on the profiling build.  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_scale.py -m gpu -x -q -s -rf --timeout 200 \
    --timeout-method thread > gpurun_out/gate_tests.log 2>&1 || { tail -30 gpurun_out/gate_tests.log; exit 1; }
grep -E "mismatch|band|passed" gpurun_out/gate_tests.log
DCTAE_LIBRARY=_ab/libprof.so timeout -k 10 400 python -u tools/gate_probe.py ${GATE_ARGS:-} > gpurun_out/gate_probe.log 2>&1
rc=$?; cat gpurun_out/gate_probe.log | tail -30; exit $rc
