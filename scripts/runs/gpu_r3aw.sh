# Heavy-first order on / off (SF_ORDER=0) for the small configs and for members' shares, interleaved, 2 reps.
R=$PWD; OUT=$R/gpurun_out/r3aw; mkdir -p $OUT
for rep in 1 2; do
  for v in "SF_NONE=0" "SF_ORDER=0"; do
    for cfg in "c1 640 360 1.0" "c2 1280 720 0.8"; do
      set -- $cfg
      env $v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --width $2 --height $3 --K $4 > $OUT/b.json 2> $OUT/b.err || exit 1
      python3 -c "import json; j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); print('$v $1', 'frame', j['frame_ms'], 'fixed', j['fixed_camera']['frame_ms'], 'lat', j['frame_latency_ms'])"
    done
    env $v PROBE_STEPS=1000 PROBE_N=2,4,8 PROBE_SLOTS=3 PROBE_SPLITS=auto timeout -k 10 300 python3 -u scripts/share_probe.py > $OUT/p.txt 2>&1 || exit 2
    echo "$v $(grep slots $OUT/p.txt)"
  done
done
