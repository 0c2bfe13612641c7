set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6_b; mkdir -p $O
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cd $R
timeout -k 10 200 python3 tools/graph_stages.py > $O/stages.log 2>&1
