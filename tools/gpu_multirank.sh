#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: two ranks
# share the card (DCTAE_BENCH_SHARE_GPU=1; RCCL refuses a duplicate GPU, so
# this mode alone runs its collectives on gloo), launched by bench.py's own
# torchrun child.  Checks that the stats-fit exchange leaves every rank with
# PatchNorm tables bit-equal to one process fitting the same shards in rank
# order (bench line: stats_fit.tables_bit_equal_to_sequential_fit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DCTAE_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus ${RANKS:-2} --steps 5 --warmup 2 --no-cpu-baseline \
    --no-configs --no-model > gpurun_out/multirank.log 2>&1
rc=$?; tail -c 1500 gpurun_out/multirank.log; echo
[ $rc -ne 0 ] && exit $rc
grep '^{' gpurun_out/multirank.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
st = d['stats_fit']
print('ranks', d['ranks'], 'value', d['value'], 'stats_fit', json.dumps(st))
assert d['ranks']['world'] == ${RANKS:-2}
assert st.get('tables_bit_equal_to_sequential_fit') is True, st
print('multi-rank rehearsal: PatchNorm tables bit-equal to the sequential fit on every rank')"
