#!/bin/bash
# Decode iteration: decode parity subset, then the bench's config-3 decode leg
# per library option set (per-kernel times).   bash tools/gpu_dec.sh "" "dec_ipb=4" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${TESTS:-decode or roundtrip}" > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dec_tests.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/dec_tests.log; exit $rc; fi
for opts in "$@"; do
  args=""
  for o in $opts; do args="$args --opt $o"; done
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-stats --no-configs \
      $args > gpurun_out/dec_bench.log 2>&1
  rc=$?
  echo "=== [$opts] rc=$rc"
  grep '^{' gpurun_out/dec_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['decode']; print('enc', d['ms_per_step'], 'dec', e['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in e['kernels'].items()}))"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/dec_bench.log; exit $rc; fi
done
