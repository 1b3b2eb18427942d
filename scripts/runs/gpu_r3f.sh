# parity suite on the remapped builder lanes + unrolled jump convolution, LDS A/B against the previous
# build (timing + PMC), frame-less timing under rocprof
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/r3f; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
REPS=3 PMC=1 scripts/lib_ab.sh r3f/lds "" sphereflake-raytracer_amd/build/libsphereflake_hip.so sphereflake-raytracer_amd/build_base/libsphereflake_hip.so
cd /tmp && export TMPDIR=/tmp
for pf in 1 0; do
  SF_PROG_PREFETCH=$pf timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prog_$pf -o run --output-format csv -- python3 $R/scripts/prog_bench.py > $OUT/prog_$pf.log 2>&1 || exit 3
  echo "== prefetch $pf"; grep -v "^W20\|^E20" $OUT/prog_$pf.log | grep batch
  head -8 $(find $OUT/prog_$pf -name "*kernel_stats.csv") | cut -d, -f1-4
done
exit $rc
