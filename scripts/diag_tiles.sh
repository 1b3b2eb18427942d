set -e
T=${1:-diag}
mkdir -p gpurun_out/$T
timeout -k 10 120 python scripts/tile_schedule.py --out gpurun_out/$T/tt.npy > gpurun_out/$T/tt.txt 2>&1
cat gpurun_out/$T/tt.txt
scripts/prof_pmc.sh $T/pmc
python3 scripts/pmc_summary.py gpurun_out/$T/pmc/* > gpurun_out/$T/pmc_summary.txt
