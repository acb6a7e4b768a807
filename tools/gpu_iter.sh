#!/bin/bash
# Iteration run on one GPU: parity subset of the encode path, then a lean
# bench sweep (encode only) over library option sets, then rocprofv3 kernel
# stats of the default encode.  Every GPU step has its own time limit and the
# script stops at the first failure.
#   bash tools/gpu_iter.sh "opts set 1" "opts set 2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${TESTS:-preprocess or encode or roundtrip or fft_path or specialised}" > gpurun_out/iter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/iter_tests.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/iter_tests.log; exit $rc; fi
for opts in "$@"; do
  args=""
  for o in $opts; do args="$args --opt $o"; done
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-decode --no-stats \
      --no-configs --no-model $args > gpurun_out/iter_bench.log 2>&1
  rc=$?
  echo "=== [$opts] rc=$rc"
  grep '^{' gpurun_out/iter_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}))"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/iter_bench.log; exit $rc; fi
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/iprof -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-decode --no-stats --no-configs \
      --no-model > gpurun_out/iprof.log 2>&1 || { tail -20 gpurun_out/iprof.log; exit 1; }
  find gpurun_out/iprof -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -20
fi
