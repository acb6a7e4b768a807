cd $GRAFT_REPO_ROOT
for o in "" "rows_fused=0" "cols_dma=0" ""; do
  DCTAE_TEST_OPTS="$o" timeout -k 10 240 python -u -m pytest tests/test_gpu_bench_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k config4 > gpurun_out/c4_$RANDOM.log 2>&1
  rc=$?
  echo "opts [$o] rc=$rc"
  [ $rc -gt 1 ] && exit $rc
done
grep -h "AssertionError: image\|passed\|failed" gpurun_out/c4_*.log | head -20
