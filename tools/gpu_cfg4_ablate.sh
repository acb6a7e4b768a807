#!/bin/bash
# Bluestein kernel ablation on the config-4 encode: per library option set,
# rocprofv3 kernel stats of the k_bs_* kernels (profiling only; outputs invalid
# under bs_ablate).   bash tools/gpu_cfg4_ablate.sh "bs_ablate=0" "bs_ablate=2" ...
# The switches exist only in a profiling build: first (in the build container)
#   make -C dct-autoencoder_amd/csrc PROFILING=1 LIB=../../_ablate/libdctae_prof.so OBJDIR=../../_ablate/obj
# and run with DCTAE_LIBRARY=_ablate/libdctae_prof.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for opts in "$@"; do
  rm -rf gpurun_out/c4ab
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c4ab -o run --output-format csv -- \
      python3 tools/cfg4_run.py 2 $opts > gpurun_out/c4ab.log 2>&1 || { tail -20 gpurun_out/c4ab.log; exit 1; }
  echo "=== $opts"
  python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c4ab/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_bs_" in r["Name"]:
        print(f"{float(r['TotalDurationNs']) / 2e6:8.3f} ms  {r['Name'][27:50]}")
PY
done
