#!/bin/bash
# Round evidence on one GPU: the default bench line, rocprofv3 kernel stats of
# the encode bench (same command family), PMC passes over the encode, and the
# bench-readable PMC profile.  Every GPU step time-limited; stop on failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out/evidence
timeout -k 10 900 python bench.py > gpurun_out/evidence/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/evidence/bench_$TAG.log; exit 1; }
tail -c 600 gpurun_out/evidence/bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/evidence/prof -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-stats --no-configs \
    > gpurun_out/evidence/rocprof_$TAG.log 2>&1 || { tail -20 gpurun_out/evidence/rocprof_$TAG.log; exit 1; }
find gpurun_out/evidence/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/evidence/rocprof_kernel_stats_$TAG.csv \;
cut -d, -f1-4 gpurun_out/evidence/rocprof_kernel_stats_$TAG.csv | head -12
bash tools/gpu_pmc_enc.sh > gpurun_out/evidence/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/evidence/pmc_$TAG.log; exit 1; }
python3 tools/pmc_enc_summary.py gpurun_out/pmc_enc --profile gpurun_out/evidence/pmc_$TAG.json --tag $TAG
