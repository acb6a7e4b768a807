#!/bin/bash
# Uninitialised-workspace check: the config-4 bench-scale test alone, then the
# whole -m gpu suite, with DCTAE_WS_POISON=1 (workspace / staging filled with
# NaN bits before every call); then N plain suites.  Stops at rc > 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {   # name, env, pytest args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 600 python -u -m pytest "$@" -m gpu -q -rf --timeout 300 --timeout-method thread \
      > gpurun_out/pc_$name.log 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc $(tail -1 gpurun_out/pc_$name.log)"
  grep -h "^FAILED\|AssertionError: image\|raw tokens changed" gpurun_out/pc_$name.log | head -8
  [ $rc -gt 1 ] && exit $rc
  return 0
}
run c4_poison "DCTAE_WS_POISON=1" tests/test_gpu_bench_scale.py -k config4
run suite_poison "DCTAE_WS_POISON=1" tests
for i in $(seq 1 ${NPLAIN:-0}); do run suite_plain_$i "X=1" tests; done
exit 0
