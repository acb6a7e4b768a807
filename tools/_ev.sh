TAG=r04 DECODE=1 bash tools/gpu_round_evidence.sh
