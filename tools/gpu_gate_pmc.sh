#!/bin/bash
# PMC of the gate cases (tools/gate_probe.py on a profiling build): HBM-side
# bytes and L2 hits of the row / column kernels with T' in HBM (t_alias 0) and
# cache-resident (t_alias 4), rows alone (gate 1) and columns alone (gate 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export DCTAE_LIBRARY=${DCTAE_LIBRARY:-_ab/libprof_c.so}
for a in 0 4; do
  for g in 1 2; do
    OUT=gpurun_out/gate_pmc/a${a}_g${g}
    rm -rf $OUT; mkdir -p $OUT
    i=0
    for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- \
          python3 tools/gate_probe.py --steps 2 --alias $a --gates $g > $OUT/p$i.log 2>&1
      rc=$?
      echo "a=$a g=$g pass $i ($grp) rc=$rc"
      if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
    done
    python3 tools/pmc_enc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
  done
done
