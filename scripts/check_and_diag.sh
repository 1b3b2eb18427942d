set -e
bash scripts/run_check.sh
bash scripts/diag_tiles.sh d9
