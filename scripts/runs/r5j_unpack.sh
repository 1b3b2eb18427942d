#!/bin/bash
# Round 5: the workgroup-dedup index-slab unpack: its tests, then 4K rows mode under a kernel trace, v1 vs v2.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
for V in 1 0; do
  SF_UNPACK_V1=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rows4k_v$V -o run --output-format csv -- python3 $R/bench.py --mode rows --gpus 8 --width 3840 --height 2160 --K 0.22 --steps 30 --warmup 5 --no-cpu-baseline --no-extras > $OUT/rows4k_v$V.json 2> $OUT/rows4k_v$V.err
  echo "== SF_UNPACK_V1=$V"
  python3 $R/scripts/unpack_overlap.py $(find $OUT/rows4k_v$V -name "*kernel_trace.csv")
  grep -E "sf_slab_unpack" $(find $OUT/rows4k_v$V -name "*kernel_stats.csv")
  python3 -c "import json; d=json.loads(open('$OUT/rows4k_v$V.json').read().strip().splitlines()[-1]); print('frame_ms', d['frame_ms'])"
done
