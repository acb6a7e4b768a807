#!/bin/bash
# PMC passes over the transformer forward (tools/model_bench.py), one
# rocprofv3 run per counter group.  Output: gpurun_out/pmcm/p<i>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcm
mkdir -p $OUT
i=0
for grp in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY" \
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
  "FETCH_SIZE"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/model_bench.py --rows 4 --steps 1 > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
