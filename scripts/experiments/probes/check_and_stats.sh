set -e
bash scripts/run_check.sh
bash scripts/stats_run.sh st11
