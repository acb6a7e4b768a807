#!/bin/bash
# Fused-kernel check on the GPU box: bitwise parity vs the two-kernel path,
# then a bench sweep of the fused options.  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "fused" > gpurun_out/pf.log 2>&1
rc=$?
tail -3 gpurun_out/pf.log
if [ $rc -ne 0 ]; then exit $rc; fi
STEPS=${STEPS:-20} bash tools/gpu_sweep.sh "fused=0" "fused=1" "fused=1 fused_slots=1" "fused=1 fused_slots=3" \
  "fused=1 fused_debug=1"
