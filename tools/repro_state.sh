#!/bin/bash
# The config-4 full-batch test after the bench-path tests in one process (the
# state the full suite runs it in), per library build; one line per build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  unset DCTAE_LIBRARY
  [ "$lib" != default ] && export DCTAE_LIBRARY=$lib
  timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_paths.py tests/test_gpu_bench_scale.py -m gpu -q \
      --timeout 300 --timeout-method thread -k "not lfq_projections_full" ${EXTRA_K:-} > gpurun_out/repro_$(basename $lib).log 2>&1
  rc=$?
  echo "=== [$lib] rc=$rc $(tail -1 gpurun_out/repro_$(basename $lib).log)"
  grep -h "AssertionError: image\|raw tokens changed" gpurun_out/repro_$(basename $lib).log | head -3
  [ $rc -gt 1 ] && exit $rc
done
exit 0
