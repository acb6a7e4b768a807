#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel trace only;
# never combined with sys/runtime traces).  Output: gpurun_out/pmc/<group>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-stats --no-model --no-configs ${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
while [ $# -gt 0 ]; do
  grp="$1"; shift
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- $BENCH > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
