#!/bin/bash
# Round-5 evidence on one GPU, every step time-limited, stop at the first
# failure: the default bench line (as the driver runs it), rocprofv3 kernel
# stats + a kernel trace of the encode bench (inter-kernel gaps per step,
# tools/trace_gaps.py), PMC passes over the encode and decode legs
# (tools/gpu_pmc_enc.sh, summary as the bench-readable profile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
OUT=gpurun_out/evidence
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -c 300 $OUT/bench_$TAG.log; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-stats --no-configs \
    > $OUT/rocprof_$TAG.log 2>&1 || { tail -20 $OUT/rocprof_$TAG.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/rocprof_kernel_stats_$TAG.csv \;
cut -d, -f1-4 $OUT/rocprof_kernel_stats_$TAG.csv | head -14
tr=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
# the encode steps: 3 warm-up then the 10 timed k_rows512pk / k_cols512b / k_sort_pack2 triples
python3 tools/trace_gaps.py "$tr" --per-call 3 --calls 10 --first 3 --match k_rows512pk --match k_cols512b \
    --match k_sort_pack2 --json $OUT/encode_trace_gaps_$TAG.json || true
PMC_OUT=$OUT/pmc DECODE=1 bash tools/gpu_pmc_enc.sh > $OUT/pmc_$TAG.log 2>&1 || { tail -20 $OUT/pmc_$TAG.log; exit 1; }
python3 tools/pmc_enc_summary.py $OUT/pmc --profile $OUT/pmc_$TAG.json --tag $TAG | tail -12
# multi-rank rehearsal at HEAD (two ranks sharing the card, gloo collectives; tools/gpu_multirank.sh)
if [ -n "${MULTIRANK:-}" ]; then
  bash tools/gpu_multirank.sh > $OUT/multirank_$TAG.log 2>&1 || { tail -30 $OUT/multirank_$TAG.log; exit 1; }
  tail -3 $OUT/multirank_$TAG.log
  cp gpurun_out/multirank.log $OUT/multirank_bench_$TAG.log
fi
