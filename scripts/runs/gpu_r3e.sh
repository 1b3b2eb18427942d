# frame-less draws A/B (parallel jump-ahead vs single workgroup, prefetch on/off) under rocprof kernel stats,
# then the LDS PMC A/B of the masked-store build, then a bench line
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for par in 1 0; do for pf in 1 0; do
  SF_MT_PARALLEL=$par SF_PROG_PREFETCH=$pf timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prog_${par}_${pf} -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $OUT/prog_${par}_${pf}.log 2>&1 || exit 3
  echo "== parallel $par prefetch $pf"; grep -v "^W20\|^E20" $OUT/prog_${par}_${pf}.log | grep batch
  head -12 $(find $OUT/prog_${par}_${pf} -name "*kernel_stats.csv") | cut -d, -f1-4
done; done
cd $R
REPS=0 PMC=1 scripts/lib_ab.sh r3e/lds "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_x1/libsphereflake_hip.so
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 4
tail -1 $OUT/bench.json | cut -c1-600
