#!/bin/bash
# Same-box A/B of library builds / option sets on the encode AND config-3
# decode legs of the bench line.
#   bash tools/gpu_ab2.sh "<library or ->|<opt=v opt=v ...>" ...
# ("-" = the in-tree libdctae.so).  Prints encode value / ms and per-kernel
# times, then the decode's.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  lib="${spec%%|*}"; opts="${spec#*|}"
  args=""
  for o in $opts; do args="$args --opt $o"; done
  if [ "$lib" = "-" ]; then unset DCTAE_LIBRARY; else export DCTAE_LIBRARY="$lib"; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-stats \
      --no-configs --no-model $args > gpurun_out/ab2_bench.log 2>&1
  rc=$?
  echo "=== [$spec] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab2_bench.log; exit $rc; fi
  grep '^{' gpurun_out/ab2_bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); e=d['decode']
print('enc', d['value'], d['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}))
print('dec', e['value'], e['ms_per_step'], json.dumps({k:v['avg_ms'] for k,v in e['kernels'].items()}))"
done
