#!/bin/bash
# PMC passes over the encode bench only (one rocprofv3 run per counter group,
# kernel trace only), then a per-kernel summary (tools/pmc_enc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_enc}
rm -rf $OUT; mkdir -p $OUT
# DECODE=1: the config-3 decode leg runs too (its kernels land in the same passes)
DEC="--no-decode"; [ -n "${DECODE:-}" ] && DEC=""
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-stats --no-model --no-configs $DEC ${BENCH_ARGS:-}"
# CMD=...: profile another program instead (e.g. CMD="python3 tools/cfg4_run.py 1")
BENCH=${CMD:-$BENCH}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
  "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- $BENCH > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_enc_summary.py $OUT ${SUMMARY_ARGS:-} > $OUT/summary.txt; cat $OUT/summary.txt
