#!/bin/bash
# Same-box A/B of library builds over the bench's GPU legs (encode, decode,
# configs 2 / 4, LFQ projections; no CPU baseline): one summary line per run.
# Usage: bash tools/ab_full.sh <lib.so|default> ...   (each GPU step time-limited; stop at the first failure)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for lib in "$@"; do
  n=$((n+1))
  unset DCTAE_LIBRARY
  [ "$lib" != default ] && export DCTAE_LIBRARY=$lib
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-stats > gpurun_out/ab_full_$n.log 2>&1
  rc=$?
  echo "=== [$lib] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab_full_$n.log; exit $rc; fi
  grep '^{' gpurun_out/ab_full_$n.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
oc=d.get('other_configs') or {}
lq=d.get('lfq_projections') or d.get('lfq') or {}
def g(x,k): return (x or {}).get(k)
print('enc', d['ms_per_step'], 'dec', g(d.get('decode'),'ms_per_step'), 'cfg2', g(oc.get('config2'),'ms_per_step'), 'cfg4', g(oc.get('config4'),'ms_per_step'), 'lfq', json.dumps({k: (v.get('ms_per_step') if isinstance(v, dict) else v) for k, v in lq.items()})[:200])"
done
