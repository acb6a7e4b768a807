set -u
TESTS="encode_512 or sq512 or batch_encoder" bash tools/gpu_try.sh "cols512b=1" "lib=_ablate/tl2/libdctae.so" "cols512b=1" "lib=_ablate/tl2/libdctae.so" && \
DCTAE_LIBRARY=_ablate/tl2/libdctae.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "encode_512 or sq512 or batch_encoder" 2>&1 | tail -3
