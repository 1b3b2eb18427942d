# Kernel-trace profile of a short bench run (rocprofv3 --kernel-trace --stats); summary to gpurun_out/<tag>/
set -e
T=${1:-stats}
R=$PWD
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 > $R/gpurun_out/$T/bench.log 2>&1
cat $(find $R/gpurun_out/$T/prof -name "*kernel_stats.csv")
tail -1 $R/gpurun_out/$T/bench.log
