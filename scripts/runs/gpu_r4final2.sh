#!/bin/bash
# Round-4 end evidence of the build in the tree, in two calls (each within gpurun's limit):
#   part a: full -m gpu suite, smoke, PMC passes (their summary in place for the bench), the default bench line,
#           its rocprofv3 kernel trace, the driver's 20-step command, the other BASELINE configs and the
#           frame-less profiles (beside the trace and alone)
#   part b: two-rank rehearsals, the spawned 2-rank line, the lone-frame probe, a member's share at 3 / 4 frames
#           in flight, the group unpack overlap, the SSAO pass trace
# Usage: scripts/runs/gpu_r4final2.sh <tag> a|b
R=$PWD; TAG=${1:-r4final2}; PART=${2:-a}; OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "$PART" = "a" ]; then
  bash scripts/round_profile.sh $TAG; rc=$?
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || { tail -5 $OUT/bench20.err; exit 6; }
  tail -1 $OUT/bench20.json | cut -c1-300
  bash scripts/configs_bench.sh $TAG/cfg > $OUT/configs.log 2>&1 || { tail -5 $OUT/configs.log; exit 7; }
  grep -v "amdgpu\|^W20\|^E20" $OUT/configs.log | grep -E "^c[0-9]|batch|mt_"
  exit $rc
fi
if [ "$PART" = "b" ] && [ -f profiles/pmc_traffic.json ]; then
  # the bench lines again with the final bench.py (same library: part a's PMC summary, committed, applies)
  timeout -k 10 400 python -u bench.py > $OUT/bench_b.json 2> $OUT/bench_b.err || { tail -20 $OUT/bench_b.err; exit 4; }
  tail -1 $OUT/bench_b.json | cut -c1-300
  for rep in 1 2 3; do
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20_b$rep.json 2> $OUT/bench20_b.err || { tail -5 $OUT/bench20_b.err; exit 6; }
    python3 -c "import json; j=json.loads(open('$OUT/bench20_b$rep.json').read().strip().split(chr(10))[-1]); print('steps20', j['frame_ms'], j['pipeline']['fill_ms'], j['roofline']['clock_mhz_live'])"
  done
fi
bash scripts/multi_rehearsal.sh > $OUT/multi.log 2>&1 || { tail -5 $OUT/multi.log; exit 8; }
cp gpurun_out/multi/*.json $OUT/ 2>/dev/null
timeout -k 10 300 python3 -u bench.py --gpus 2 --rehearse --steps 40 --warmup 5 > $OUT/spawn2.json 2> $OUT/spawn2.err || { tail -5 $OUT/spawn2.err; exit 9; }
SF_FLAGS=0x20 timeout -k 10 120 python3 -u scripts/latency_probe.py > $OUT/latency.txt 2>&1 || { tail -5 $OUT/latency.txt; exit 10; }
PROBE_STEPS=600 PROBE_N=1,2,4,8 PROBE_SLOTS=3,4 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/share_probe.txt 2>&1 || { tail -3 $OUT/share_probe.txt; exit 11; }
grep slots $OUT/share_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rows8 -o run --output-format csv -- python3 $R/bench.py --mode rows --gpus 8 --steps 60 --warmup 5 --no-cpu-baseline > $OUT/rows8.log 2>&1 || { tail -5 $OUT/rows8.log; exit 12; }
python3 $R/scripts/unpack_overlap.py $(find $OUT/rows8 -name "*kernel_trace.csv") | tee $OUT/rows8_overlap.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/post -o run --output-format csv -- python3 $R/scripts/post_probe.py > $OUT/post.log 2>&1 || { tail -5 $OUT/post.log; exit 13; }
grep "post " $OUT/post.log
