set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh test || exit $?
bash tools/gpu_sweep.sh "chunk_bytes=1e12 rows_prefetch=1" "chunk_bytes=1e12" "chunk_bytes=400e6 rows_prefetch=1"
