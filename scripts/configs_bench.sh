#!/bin/bash
# Bench lines of the other BASELINE configs (c1, c2, c4, c5) + a rocprof kernel-stats run of the
# frame-less mode. Usage (on the box, repo root): scripts/configs_bench.sh <tag>
set -e
OUT=gpurun_out/${1:-cfg}; mkdir -p $OUT
R=$PWD
for cfg in "c1 640 360 1.0" "c2 1280 720 0.8" "c4 3840 2160 0.22"; do
  set -- $cfg
  timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 > $OUT/bench_$1.json 2> $OUT/bench_$1.err
  python3 -c "import json; j=json.loads(open('$OUT/bench_$1.json').read().strip().split(chr(10))[-1]); print('$1', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'check', j['check']['bit_exact'], 'Mrays', j['value'], 'fixed', j['fixed_camera']['frame_ms'], 'depth', j['config']['max_depth'])"
done
timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-extras --width 16384 --height 16384 --K 0.2 --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
python3 -c "import json; j=json.loads(open('$OUT/bench_c5.json').read().strip().split(chr(10))[-1]); print('c5', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'check', j['check']['bit_exact'], 'Mrays', j['value'], 'fixed', j['fixed_camera']['frame_ms'], 'depth', j['config']['max_depth'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$OUT/frameless -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $R/$OUT/frameless.log 2>&1
cat $R/$OUT/frameless.log | grep -v amdgpu
cat $(find $R/$OUT/frameless -name "*kernel_stats.csv")
# the frame-less draws alone: without the prefetch (SF_PROG_PREFETCH=0) each batch's draw kernels run on the
# context stream ahead of its trace, not beside the previous batch's trace -- their durations unshared
SF_PROG_PREFETCH=0 PROG_BATCHES=262144 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$OUT/frameless_alone -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $R/$OUT/frameless_alone.log 2>&1
cat $(find $R/$OUT/frameless_alone -name "*kernel_stats.csv") | grep -i "mt_\|Name"
