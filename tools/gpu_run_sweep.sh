set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh test || exit $?
bash tools/gpu_sweep.sh "chunk_bytes=1e12 rows_prefetch=1" "chunk_bytes=1e12 rows_prefetch=1 xcd_order=0" "chunk_bytes=1e12 rows_prefetch=1 t_layout=1" "rows_prefetch=1 chunk_bytes=200e6"
