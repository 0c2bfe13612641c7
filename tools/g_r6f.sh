set -o pipefail
export TAG=r6f C2_ONLY=1
bash tools/sessions/final_r6.sh bench > gpurun_out/r6f_bench.txt 2>&1 && bash tools/sessions/final_r6.sh cache > gpurun_out/r6f_cache.txt 2>&1 && bash tools/sessions/final_r6.sh prof > gpurun_out/r6f_prof.txt 2>&1
