set -e
mkdir -p gpurun_out/r5h
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace -d $GRAFT_REPO_ROOT/gpurun_out/r5h/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/host_overhead_probe.py 12 > $GRAFT_REPO_ROOT/gpurun_out/r5h/probe.txt 2>&1
cat $GRAFT_REPO_ROOT/gpurun_out/r5h/probe.txt
ls -R $GRAFT_REPO_ROOT/gpurun_out/r5h/tr | head
