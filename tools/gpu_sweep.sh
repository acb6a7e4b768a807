#!/bin/bash
# Option sweep of bench.py on the GPU box (one process per configuration).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for opts in "$@"; do
  args=""
  for o in $opts; do args="$args --opt $o"; done
  echo "=== $opts"
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $args > gpurun_out/sweep.log 2>&1
  rc=$?
  grep '^{' gpurun_out/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}))"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
