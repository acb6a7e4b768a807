#!/bin/bash
# GPU-box validation run: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (exit >= 124 or a
# signal) stops the script so nothing else touches the GPU after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "FATAL: $name rc=$rc, stopping"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 900 python -m pytest tests -m gpu -q -rA
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps ${STEPS:-10} --warmup 3
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing
  find $OUT/prof -name "*stats*" | head
fi
