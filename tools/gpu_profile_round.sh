# Round evidence: default bench line, rocprofv3 kernel stats of the same
# command, PMC traffic passes.  Each GPU step time-limited; stop on a crash.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-stats --no-model --no-configs > gpurun_out/rocprof.log 2>&1 || exit $?
bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
