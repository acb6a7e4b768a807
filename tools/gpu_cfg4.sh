#!/bin/bash
# Config-4 (ragged) iteration: Bluestein / large-ragged parity subset, then
# rocprofv3 kernel stats of the config-4 encode (tools/cfg4_run.py).
#   bash tools/gpu_cfg4.sh [library options key=value ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${TESTS:-bluestein or large_ragged}" > gpurun_out/c4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c4_tests.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/c4_tests.log; exit $rc; fi
rm -rf gpurun_out/c4prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run --output-format csv -- \
    python3 tools/cfg4_run.py 3 "$@" > gpurun_out/c4prof.log 2>&1 || { tail -20 gpurun_out/c4prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c4prof/**/*kernel_stats.csv", recursive=True)[0]
tot = 0.0
for r in csv.DictReader(open(f)):
    if "k_synth" in r["Name"] or "rocclr" in r["Name"]:
        continue
    ms = float(r["TotalDurationNs"]) / 1e6 / 3
    tot += ms
    print(f"{ms:8.3f} ms  {r['Name'][:90]}")
print(f"{tot:8.3f} ms  total per encode")
PY
