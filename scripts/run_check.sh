set -e
T=${1:-v20}
mkdir -p gpurun_out/$T
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash scripts/count_probe.sh
scripts/sweep.sh ${T}sw "SF_FLAGS=0" "SF_FLAGS=1" "SF_FLAGS=0"
timeout -k 10 120 python scripts/tile_schedule.py --reps 2 --out gpurun_out/$T/tt.npy > gpurun_out/$T/tt.txt 2>&1
grep -v amdgpu gpurun_out/$T/tt.txt
python3 scripts/sched_sim.py gpurun_out/$T/tt.npy 7168
