#!/bin/bash
# End-of-round check: config-4 run-to-run stress (default library, then an
# optional A/B library), the -m gpu suite, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
unset DCTAE_LIBRARY
timeout -k 10 200 python -u tools/c4_stress.py ${NSTRESS:-150} "" > gpurun_out/chk_stress.log 2>&1 || exit 11
grep -v amdgpu.ids gpurun_out/chk_stress.log | grep -v "^    " | tail -4
if [ -n "$ABLIB" ]; then
  DCTAE_LIBRARY=$PWD/$ABLIB timeout -k 10 200 python -u tools/c4_stress.py 100 "" > gpurun_out/chk_stress_ab.log 2>&1 || exit 12
  echo "AB $ABLIB:"; grep -v amdgpu.ids gpurun_out/chk_stress_ab.log | grep -v "^    " | tail -4
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/chk_tests.log 2>&1
rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/chk_tests.log)"; grep "^FAILED" gpurun_out/chk_tests.log | head
[ $rc -gt 1 ] && exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 600 python -u bench.py > gpurun_out/chk_bench.log 2>&1 || exit 13
tail -1 gpurun_out/chk_bench.log | cut -c1-600
