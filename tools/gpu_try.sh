#!/bin/bash
# Iteration: parity tests selected by TESTS (pytest -k), then a same-box A/B of
# the encode bench over option sets ("opt=v opt=v" per argument; a leading
# "lib=<path>" selects another libdctae.so build).  DEC=1 adds the config-3
# decode leg; CFG2=1 / CFG4=1 time config 2 / 4 only (tools/cfg2_try.py, cfg4_try.py).  Each GPU step time-limited; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${TFILES:-tests/test_gpu_parity.py} -m gpu -x -q -rf --timeout 200 \
      --timeout-method thread -k "$TESTS" > gpurun_out/try_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/try_tests.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|error" gpurun_out/try_tests.log | head -40; exit $rc; fi
fi
for opts in "$@"; do
  args=""
  unset DCTAE_LIBRARY
  for o in $opts; do
    case $o in lib=*) export DCTAE_LIBRARY="${o#lib=}";; *) args="$args --opt $o";; esac
  done
  if [ -n "${LFQP:-}" ]; then   # the LFQ-projection leg only (tools/lfqp_try.py)
    timeout -k 10 300 python tools/lfqp_try.py $args > gpurun_out/try_lfqp.log 2>&1
    rc=$?; echo "=== lfqp [$opts] rc=$rc"; tail -1 gpurun_out/try_lfqp.log
    [ $rc -ne 0 ] && exit $rc
    continue
  fi
  if [ -n "${CFG4:-}" ]; then   # config 4 only (tools/cfg4_try.py)
    timeout -k 10 300 python tools/cfg4_try.py $args > gpurun_out/try_cfg4.log 2>&1
    rc=$?; echo "=== cfg4 [$opts] rc=$rc"; tail -1 gpurun_out/try_cfg4.log
    [ $rc -ne 0 ] && exit $rc
    continue
  fi
  if [ -n "${CFG2:-}" ]; then   # config 2 only (tools/cfg2_try.py)
    timeout -k 10 200 python tools/cfg2_try.py $args > gpurun_out/try_cfg2.log 2>&1
    rc=$?; echo "=== cfg2 [$opts] rc=$rc"; tail -1 gpurun_out/try_cfg2.log
    [ $rc -ne 0 ] && exit $rc
    continue
  fi
  dec="--no-decode"; [ -n "${DEC:-}" ] && dec=""
  timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline $dec --no-stats \
      --no-configs --no-model $args > gpurun_out/try_bench.log 2>&1
  rc=$?
  echo "=== [$opts] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/try_bench.log; exit $rc; fi
  grep '^{' gpurun_out/try_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}), json.dumps({k: v.get('avg_ms') for k, v in (d.get('decode') or {}).get('kernels', {}).items()}), (d.get('decode') or {}).get('ms_per_step'))"
done
