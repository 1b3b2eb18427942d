#!/bin/bash
# Round-6 evidence pass on one GPU box (repo root): the full GPU parity suite, smoke, the PMC passes of the 1080p
# bench (profiles/pmc_traffic.json for this library: the bench lines of this run and of the driver read it), the default
# bench line (200 steps) and three driver-shaped 20-step lines, a kernel-trace (--stats) profile of the default bench
# command, the other BASELINE configs, the index-slab unpack alone and the members' shares.
# Every GPU step has its own time limit; the script stops at the first failure. Usage: round6_evidence.sh <tag>
set -e
TAG=${1:-r6end}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
sha256sum sphereflake-raytracer_amd/build/libsphereflake_hip.so > $OUT/lib_sha256.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
scripts/prof_pmc.sh $TAG/pmc
python3 scripts/pmc_summary.py --json $OUT/pmc_traffic.json --config "1920x1080 K=0.25 moving" $OUT/pmc/*/ > $OUT/pmc_summary.txt
cp $OUT/pmc_traffic.json $R/profiles/pmc_traffic.json
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $OUT/bench20_$i.json 2> $OUT/bench20_$i.err
done
for f in $OUT/bench.json $OUT/bench20_1.json $OUT/bench20_2.json $OUT/bench20_3.json; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); p=d['pipeline']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'steady', p['steady_frame_ms'], 'fill', p['fill_ms'], 'lat', d['frame_latency_ms'], 'clk', d['roofline']['clock_mhz_live'], 'frac', d['roofline']['frac'], 'exact', d['check']['bit_exact'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $R/bench.py > $OUT/stats_bench.json 2> $OUT/stats.log
cp $(find $OUT/stats -name "*kernel_stats.csv") $OUT/kernel_stats.csv
head -6 $OUT/kernel_stats.csv
cd $R
for cfg in "c1 640 360 1.0" "c2 1280 720 0.8" "c4 3840 2160 0.22"; do
  set -- $cfg
  timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 > $OUT/bench_$1.json 2> $OUT/bench_$1.err
  python3 -c "import json; j=json.loads(open('$OUT/bench_$1.json').read().strip().split(chr(10))[-1]); print('$1', 'frame', j['frame_ms'], 'steady', j['pipeline']['steady_frame_ms'], 'lat', j['frame_latency_ms'], 'check', j['check']['bit_exact'], 'Mrays', j['value'])"
done
timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-extras --width 16384 --height 16384 --K 0.2 --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
python3 -c "import json; j=json.loads(open('$OUT/bench_c5.json').read().strip().split(chr(10))[-1]); print('c5', 'frame', j['frame_ms'], 'check', j['check']['bit_exact'], 'Mrays', j['value'])"
for W in "3840 2160 0.22" "1920 1080 0.25"; do
  timeout -k 10 200 python3 -u scripts/unpack_probe.py $W 8 50 2>&1 | grep unpack | tee -a $OUT/unpack.txt
done
timeout -k 10 300 python3 -u scripts/share_probe.py 1920 1080 0.25 2>&1 | grep -v amdgpu.ids | tee -a $OUT/share.txt
# the driver's N > 1 flow rehearsed on this box's one GPU (two self-spawned ranks; every leg but the RCCL gather)
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rehearse2.json 2> $OUT/rehearse2.err
python3 -c "import json; d=json.loads(open('$OUT/rehearse2.json').read().strip().splitlines()[-1]); print('rehearse2', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['check']['bit_exact'])" | tee $OUT/rehearse2.txt
