# Jump-ahead windows split over 8 / 16 / 32 workgroups: frame-less parity (draw tests) per build, batch times,
# rocprof kernel stats.
R=$PWD; OUT=$R/gpurun_out/r3v; mkdir -p $OUT
for b in build build_p16 build_p32; do
  L=$R/sphereflake-raytracer_amd/$b/libsphereflake_hip.so
  SF_LIB=$L timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "progressive or mt or initialize" --timeout 120 --timeout-method thread > $OUT/pytest_$b.log 2>&1; rc=$?
  echo "== $b: $(tail -1 $OUT/pytest_$b.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
  SF_LIB=$L timeout -k 10 120 python3 -u scripts/prog_bench.py 2>&1 | grep -v amdgpu | grep 262144 || exit 2
  cd /tmp && export TMPDIR=/tmp
  SF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$b -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $OUT/prof_$b.log 2>&1 || exit 3
  grep "sf_mt\|progressive_trace\|packet" $(find $OUT/prof_$b -name "*kernel_stats.csv") | cut -d, -f1-4
  cd $R
done
