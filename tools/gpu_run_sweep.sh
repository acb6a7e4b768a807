set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh test || exit $?
bash tools/gpu_sweep.sh "" "chunk_bytes=64e6" "chunk_bytes=320e6" "chunk_bytes=1e12"
