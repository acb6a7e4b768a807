set -u
TESTS="encode_512 or sq512 or batch_encoder or specialised" bash tools/gpu_try.sh "cols512b=1" "lib=_ablate/tl1/libdctae.so" "lib=_ablate/tl2/libdctae.so" "lib=_ablate/tl3/libdctae.so" "cols512b=1" "lib=_ablate/tl2/libdctae.so" "lib=_ablate/tl3/libdctae.so"
