#!/bin/bash
# Same-box A/B of library builds / option sets on the encode bench line.
#   bash tools/gpu_ab.sh "<library or ->|<opt=v opt=v ...>" ...
# ("-" = the in-tree libdctae.so).  Each run: bench.py encode only, STEPS steps;
# prints value, ms/step and per-kernel device times.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  lib="${spec%%|*}"; opts="${spec#*|}"
  args=""
  for o in $opts; do args="$args --opt $o"; done
  if [ "$lib" = "-" ]; then unset DCTAE_LIBRARY; else export DCTAE_LIBRARY="$lib"; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-decode --no-stats \
      --no-configs --no-model $args > gpurun_out/ab_bench.log 2>&1
  rc=$?
  echo "=== [$spec] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab_bench.log; exit $rc; fi
  grep '^{' gpurun_out/ab_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}))"
done
