#!/bin/bash
# End-of-round evidence on one GPU: the GPU test suite, smoke(), the default
# bench line + rocprofv3 kernel stats + PMC passes (tools/gpu_profile_round.sh)
# and the transformer forward's rocprofv3 kernel stats.  Every GPU step has
# its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -30 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash tools/gpu_profile_round.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o run --output-format csv -- \
    python3 tools/model_bench.py > gpurun_out/mprof.log 2>&1 || { tail -20 gpurun_out/mprof.log; exit 1; }
echo "model profile ok"
