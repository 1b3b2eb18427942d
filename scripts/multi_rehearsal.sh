# Two ranks on the one GPU of a gpurun box, gloo backend: rehearses bench.py's multi-rank flow
# (barriers, max-over-ranks timing, row-band gather) that the driver runs over RCCL on 8 GPUs.
set -e
mkdir -p gpurun_out/multi
export SF_BENCH_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/multi/frames.json 2> gpurun_out/multi/frames.err \
    || { tail -20 gpurun_out/multi/frames.err; exit 1; }
cat gpurun_out/multi/frames.json
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
    bench.py --gpus 2 --steps 10 --warmup 3 --mode rows --no-cpu-baseline > gpurun_out/multi/rows.json 2> gpurun_out/multi/rows.err \
    || { tail -20 gpurun_out/multi/rows.err; exit 1; }
cat gpurun_out/multi/rows.json
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
    bench.py --gpus 2 --steps 10 --warmup 3 --mode rows-rccl --no-cpu-baseline > gpurun_out/multi/rows_rccl.json 2> gpurun_out/multi/rows_rccl.err \
    || { tail -20 gpurun_out/multi/rows_rccl.err; exit 1; }
cat gpurun_out/multi/rows_rccl.json
