#!/bin/bash
# Round 4: the order variant that won on 1080p (order on, rebuilt every 16th render from that render's costs only,
# model splits) against the current defaults on the other BASELINE configs; the SSAO consumer's profile (kernel
# trace + PMC); the index unpack's cost after the centre-only last level.
R=$PWD; OUT=$R/gpurun_out/r4c; mkdir -p $OUT
run() {  # run <name> <steps> <w> <h> <K> <env...>
  local name=$1 steps=$2 w=$3 h=$4 k=$5; shift 5
  env "$@" timeout -k 10 200 python3 -u bench.py --steps $steps --warmup 5 --width $w --height $h --K $k --no-cpu-baseline --no-extras > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "
import json; j=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); p=j.get('pipeline',{})
print('%-12s steps %3d frame %.4f steady %.4f lat %.4f fixed %.4f check %s' % ('$name', $steps, j['ms_per_step'], p.get('steady_frame_ms',0), j['frame_latency_ms'], j['fixed_camera']['frame_ms'], j.get('check',{}).get('bit_exact')))"
}
NEW="SF_ORDER=1 SF_ORDER_EVERY=16 SF_ORDER_RECORD=0 SF_SPLIT_BUCKETS=model"
for rep in 1 2; do
  for cfg in "c2 1280 720 0.8" "c4 3840 2160 0.22"; do
    set -- $cfg
    for steps in 20 200; do
      run ${1}_base_$steps $steps $2 $3 $4 SF_NOP=1 || exit 1
      run ${1}_new_$steps $steps $2 $3 $4 $NEW || exit 1
    done
  done
  run c5_base_10 10 16384 16384 0.2 SF_NOP=1 || exit 1
  run c5_new_10 10 16384 16384 0.2 $NEW || exit 1
  run c3_base_20 20 1920 1080 0.25 SF_NOP=1 || exit 1
  run c3_new_20 20 1920 1080 0.25 $NEW || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/post -o run --output-format csv -- python3 $R/scripts/post_probe.py > $OUT/post.log 2>&1 || { tail -5 $OUT/post.log; exit 2; }
grep post $OUT/post.log; grep -E "sf_post|Name" $(find $OUT/post -name "*kernel_stats.csv") | cut -d, -f1-4
for pass in "pm1 FETCH_SIZE" "pm2 WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "pm3 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS" "pm4 GRBM_GUI_ACTIVE GRBM_COUNT"; do
  set -- $pass; name=$1; shift
  POST_REPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/post_$name -o run --output-format csv -- python3 $R/scripts/post_probe.py > $OUT/post_$name.log 2>&1 || echo "pmc $name failed"
done
cd $R
timeout -k 10 200 python3 -u bench.py --mode rows --gpus 8 --steps 60 --warmup 5 --no-cpu-baseline > $OUT/rows8.json 2> $OUT/rows8.err || { tail -5 $OUT/rows8.err; exit 3; }
tail -1 $OUT/rows8.json | cut -c1-300
# frame-less leg: the standalone probe vs the bench process's leg, prefetch stream at normal / greatest priority
timeout -k 10 120 python3 -u scripts/prog_bench.py > $OUT/prog_bench.txt 2>&1 || exit 4
grep "262144" $OUT/prog_bench.txt
for v in 0 1; do
  SF_PF_PRIO=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/fl$v.json 2> $OUT/fl$v.err || { tail -5 $OUT/fl$v.err; exit 5; }
  python3 -c "import json; j=json.loads(open('$OUT/fl$v.json').read().strip().splitlines()[-1]); print('pf_prio=$v', j['frameless'])"
done
# a member's share (rank 0's bands of an 8-way split, 3 frames in flight): in-wave tie re-trace vs the fixup launch,
# and the heavy-first order with model splits (rebuilt every 16th render)
for v in "base SF_NOP=1" "fixup SF_TIE_INLINE=0" "ord16m SF_ORDER=1 SF_ORDER_EVERY=16 SF_ORDER_RECORD=0" "ord16m4 SF_ORDER=1 SF_ORDER_EVERY=16 SF_ORDER_RECORD=0 SF_SPLIT_PARTS=4"; do
  set -- $v; name=$1; shift
  env "$@" PROBE_STEPS=600 PROBE_N=1,8 PROBE_SLOTS=3 PROBE_SPLITS=auto,model timeout -k 10 200 python3 -u scripts/share_probe.py > $OUT/share_$name.txt 2>&1 || { tail -3 $OUT/share_$name.txt; exit 6; }
  echo "$name: $(grep slots $OUT/share_$name.txt | tr '\n' ' ')"
done
