#!/bin/bash
# MALL-residency sweep: chunk sizes (T of a chunk kept in the Infinity Cache) x T layout
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_sweep.sh "chunk_bytes=1e12" "chunk_bytes=32e6" "chunk_bytes=64e6" "chunk_bytes=128e6" "chunk_bytes=200e6" \
  "t_layout=1" "chunk_bytes=64e6 t_layout=1" "chunk_bytes=128e6 t_layout=1"
