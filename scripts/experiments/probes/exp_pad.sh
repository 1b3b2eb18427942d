set -e
for v in "" "SF_LIB=$PWD/sphereflake-raytracer_amd/build_pad8/libsphereflake_hip.so" "" "SF_LIB=$PWD/sphereflake-raytracer_amd/build_pad8/libsphereflake_hip.so"; do
  env $v timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 30 > gpurun_out/pad.json
  python3 -c "import json; j=json.loads(open('gpurun_out/pad.json').read().strip().split(chr(10))[-1]); print('${v:-base}'[-40:], j['frame_ms'], j['roofline']['kernel_ms'])"
done
