#!/bin/bash
# Round-4 evidence of the build in the tree: full suite, smoke, the default bench line and the driver's command,
# rocprofv3 kernel trace of the bench, the PMC passes (recorded with the library build in pmc_traffic.json), the
# other BASELINE configs and the frame-less profile, the two-rank rehearsals, the lone-frame probe, the group
# unpack overlap. Each GPU step has its own limit; a failing step ends the script.
R=$PWD; TAG=${1:-r4final}; OUT=$R/gpurun_out/$TAG
bash scripts/round_profile.sh $TAG; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || { tail -5 $OUT/bench20.err; exit 6; }
tail -1 $OUT/bench20.json | cut -c1-400
bash scripts/configs_bench.sh $TAG/cfg > $OUT/configs.log 2>&1 || { tail -5 $OUT/configs.log; exit 7; }
grep -v "amdgpu\|^W20\|^E20" $OUT/configs.log | grep -E "^c[0-9]|batch"
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
exit $rc
