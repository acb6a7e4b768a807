#!/bin/bash
# Round-5 GPU session: full GPU suite, then the same-box A/Bs named in $AB
# (tools/gpu_try.sh argument sets, DEC=1 for the decode leg), then the config-2
# kernel trace (20 back-to-back BatchEncoder calls under rocprofv3
# --kernel-trace, gaps by tools/trace_gaps.py).  Every GPU step time-limited;
# stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${TSEL:-} \
      > gpurun_out/r5_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/r5_tests.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/r5_tests.log | head -30; exit $rc; fi
fi
if [ -n "${AB:-}" ]; then
  eval "bash tools/gpu_try.sh $AB" || exit 1
fi
if [ -n "${PROBE:-}" ]; then   # DFT16 on VALU vs MFMA (tools/probe/dft16_mfma.hip) + its counters
  timeout -k 10 120 ./tools/probe/dft16_mfma > gpurun_out/dft16_probe.json 2> gpurun_out/dft16_probe.err || { cat gpurun_out/dft16_probe.err; exit 1; }
  cat gpurun_out/dft16_probe.json
  rm -rf gpurun_out/dft16_pmc
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES \
      SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/dft16_pmc -o pmc -- ./tools/probe/dft16_mfma \
      > gpurun_out/dft16_pmc.log 2>&1 || { tail -20 gpurun_out/dft16_pmc.log; exit 1; }
fi
if [ -n "${CFG2TRACE:-}" ]; then
  rm -rf gpurun_out/cfg2trace
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/cfg2trace -o run --output-format csv -- \
      python3 tools/cfg2_try.py --steps 20 --no-kernel-timing > gpurun_out/cfg2trace.log 2>&1 || { tail -20 gpurun_out/cfg2trace.log; exit 1; }
  tail -1 gpurun_out/cfg2trace.log
  f=$(find gpurun_out/cfg2trace -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_gaps.py "$f" --per-call 3 --calls 20 --json gpurun_out/cfg2_gaps.json || exit 1
fi
