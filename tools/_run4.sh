set -u
bash tools/gpu_try.sh "cols512b=1" "lib=_ablate/tstrip/libdctae.so" "lib=_ablate/abl1/libdctae.so" "lib=_ablate/abl3/libdctae.so" "lib=_ablate/abl4/libdctae.so" "lib=_ablate/abl5/libdctae.so" "lib=_ablate/prof/libdctae.so t_alias=8" "cols512b=0" "lib=_ablate/tstrip/libdctae.so" && \
BENCH_ARGS="" PMC_OUT=gpurun_out/pmc_r04a bash tools/gpu_pmc_enc.sh > gpurun_out/pmc_r04a.log 2>&1; tail -30 gpurun_out/pmc_r04a.log
