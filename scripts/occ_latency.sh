# Diagnostics: tile latency vs co-residency (persistent grid capped by SF_MAX_BLOCKS, 2 waves/block)
set -e
mkdir -p gpurun_out/lat
for B in 128 512 1024 2048 0; do
  SF_MAX_BLOCKS=$B timeout -k 10 120 python scripts/tile_schedule.py --reps 2 --out gpurun_out/lat/b$B.npy > gpurun_out/lat/b$B.txt 2>&1
  echo "blocks=$B $(tail -1 gpurun_out/lat/b$B.txt)"
done
