#!/bin/bash
# The full -m gpu suite once per library build (in order), one line each;
# stops at a build whose suite errors out (rc > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for lib in "$@"; do
  n=$((n+1))
  unset DCTAE_LIBRARY
  [ "$lib" != default ] && export DCTAE_LIBRARY=$lib
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
      > gpurun_out/suite_$n.log 2>&1
  rc=$?
  echo "=== [$lib] rc=$rc $(tail -1 gpurun_out/suite_$n.log)"
  grep -h "^FAILED\|AssertionError: image\|raw tokens changed" gpurun_out/suite_$n.log | head -5
  [ $rc -gt 1 ] && exit $rc
done
exit 0
