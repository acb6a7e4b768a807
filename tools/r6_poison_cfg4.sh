cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
DCTAE_WS_POISON=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/chk_poison.log 2>&1; rc=$?
echo "poison suite rc=$rc $(tail -1 gpurun_out/chk_poison.log)"; grep "^FAILED" gpurun_out/chk_poison.log | head
[ $rc -gt 1 ] && exit $rc
CFG4=1 tools/gpu_try.sh "" "lib=$PWD/_ab/pipew0.so" "" "lib=$PWD/_ab/pipew0.so" || exit 21
rm -rf gpurun_out/prof_cfg4b; timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg4b -o run -- python3 tools/cfg4_run.py 3 > gpurun_out/prof_cfg4b.log 2>&1 || exit 22
find gpurun_out/prof_cfg4b -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-200
