set -o pipefail
mkdir -p gpurun_out/r6d
TSPLAT_LIB=tools/wastamp_tmp.so timeout -k 10 120 python tools/wa_stamps.py --x3 > gpurun_out/r6d/stamps_v2.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 TSPLAT_LIB=tools/wastamp_tmp.so timeout -k 10 120 python tools/wa_stamps.py --x3 > gpurun_out/r6d/stamps_v1.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 > gpurun_out/r6d/wa.log 2>&1 && \
TSPLAT_WINATTN_X3_PRIO=0 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6d/wa.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 >> gpurun_out/r6d/wa.log 2>&1 && \
timeout -k 10 120 python tools/bench_winattn.py --dtype x3 --batch 16 >> gpurun_out/r6d/wa.log 2>&1 && \
TSPLAT_WINATTN_X3=v1 timeout -k 10 120 python tools/bench_winattn.py --dtype x3 --batch 16 >> gpurun_out/r6d/wa.log 2>&1
