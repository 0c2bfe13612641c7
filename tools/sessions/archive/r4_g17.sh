#!/bin/bash
# Round 4: XCD-aware (tile block, output block) order in the bf16x3 Winograd kernel: kernel tests,
# census, FETCH / WRITE of the 163 -> 168 conv, C2 x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-r4_g17}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv.py -k "bf16x3" -m gpu > $OUT/pytest_w3.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_w3.log | head; tail -3 $OUT/pytest_w3.log; exit 1; }
tail -1 $OUT/pytest_w3.log
timeout -k 10 400 python -u tools/bench_wino3.py > $OUT/bench_wino3.log 2>&1 || { tail -3 $OUT/bench_wino3.log; exit 2; }
grep -v amdgpu $OUT/bench_wino3.log | tail -26
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_w3_$C -o run --output-format csv -- python3 $R/tools/one_wino3.py 2 163 168 256 256 > $OUT/pmc_w3_$C.log 2>&1 || exit 3
done
cd $R
f() { find $OUT/$1 -name "*counter_collection.csv" | head -1; }
python3 tools/pmc_traffic.py $(f pmc_w3_FETCH_SIZE) $(f pmc_w3_WRITE_SIZE) conv_kernel $OUT/traffic_wino3_163x168_b1.json | cut -c1-200
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2_$i.log 2>&1 || { tail -5 $OUT/bench_c2_$i.log; exit 5; }
  echo "c2 $i $(tail -1 $OUT/bench_c2_$i.log | cut -c1-120)"
done
timeout -k 10 300 python -u bench.py --batch 8 --dense-dtype bf16x3 --attn-dtype bf16 --no-cpu-baseline > $OUT/bench_c3_stated.log 2>&1 || { tail -5 $OUT/bench_c3_stated.log; exit 6; }
echo "c3 stated $(tail -1 $OUT/bench_c3_stated.log | cut -c1-120)"
