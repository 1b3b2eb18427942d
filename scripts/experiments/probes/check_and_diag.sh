set -e
bash scripts/run_check.sh
bash scripts/stats_run.sh ${1:-st}
bash scripts/diag_tiles.sh ${2:-d}
