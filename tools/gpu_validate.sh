#!/bin/bash
# Full validation on one GPU: the -m gpu suite, smoke(), the default bench line.
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/val_tests.log 2>&1
rc=$?; tail -5 gpurun_out/val_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/val_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val_smoke.log 2>&1 || { tail -30 gpurun_out/val_smoke.log; exit 1; }
tail -2 gpurun_out/val_smoke.log
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/val_bench.log 2>&1 || { tail -30 gpurun_out/val_bench.log; exit 1; }
  grep '^{' gpurun_out/val_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['roofline']), json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}), json.dumps(d.get('other_configs')), json.dumps({k: d['decode'].get(k) for k in ('value','ms_per_step','hbm_roofline_frac')}))"
fi
