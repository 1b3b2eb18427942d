# rocprofv3 kernel stats: bench with SF_ORDER=0 vs 1, and the tile_schedule script (4 renders)
set -e
R=$PWD
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp
for O in 0 1; do
  SF_ORDER=$O timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab/o$O -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 > $R/gpurun_out/ab/o$O.log 2>&1
  echo "== SF_ORDER=$O"; grep -h "sf_" $(find $R/gpurun_out/ab/o$O -name "*kernel_stats.csv")
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ab/ts -o run --output-format csv -- python3 $R/scripts/tile_schedule.py --out $R/gpurun_out/ab/tt.npy > $R/gpurun_out/ab/ts.log 2>&1
python3 - <<'PY'
import csv,glob
f=glob.glob('/root/repo/gpurun_out/ab/ts/**/*kernel_trace.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Kernel_Name'].startswith('sf_'): print(r['Kernel_Name'], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3, 'us')
PY
