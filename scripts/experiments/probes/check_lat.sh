set -e
bash scripts/run_check.sh
bash scripts/stats_run.sh ${1:-st}
bash scripts/occ_latency.sh
