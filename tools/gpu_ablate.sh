#!/bin/bash
# Ablation timing of the column kernel: builds variants with parts skipped
# (-DDCTAE_ABLATE=mask: columns 1 load, 2 pass 1, 4 pass 2, 8 post, 16 epilogue;
# rows 32 no T stores, 64 no RGB loads) and
# benches each through DCTAE_LIBRARY (results are wrong; only timings matter).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out _ablate
if [ "${BUILD:-0}" = 1 ]; then
  cd dct-autoencoder_amd/csrc
  for m in "$@"; do
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -std=c++17 -ffp-contract=off -DDCTAE_ABLATE=$m \
      -o ../../_ablate/libdctae_$m.so dctae_kernels.hip dctae_fft.hip dctae_fft2.hip dctae_idct.hip dctae_vq.hip dctae_stats.hip dctae_model.hip dctae_api.hip || exit 1
  done
  cd ../..
fi
for m in "$@"; do
  echo "=== ablate $m"
  DCTAE_LIBRARY=$PWD/_ablate/libdctae_$m.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${ABL_OPTS:-} > gpurun_out/ablate.log 2>&1
  rc=$?
  grep '^{' gpurun_out/ablate.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps({k:v['avg_ms'] for k,v in d['kernels'].items()}))"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ablate.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
