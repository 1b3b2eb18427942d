# Two ranks on the one GPU of a gpurun box (gloo control plane): rehearses bench.py's multi-rank flow -- the
# driver's default `--gpus 2` command with --rehearse (every leg but the RCCL gather, which RCCL refuses on a
# shared device), the weak-scaling frames mode and the one-process group mode.
set -e
mkdir -p gpurun_out/multi
run() {  # run <name> <port> <bench args...>
  local name=$1 port=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 2 "$@" > gpurun_out/multi/$name.json 2> gpurun_out/multi/$name.err \
      || { tail -20 gpurun_out/multi/$name.err; exit 1; }
  cat gpurun_out/multi/$name.json
}
run dist 29517 --steps 40 --warmup 5 --rehearse
run frames 29518 --steps 20 --warmup 3 --mode frames --no-cpu-baseline --no-extras
run rows 29519 --steps 20 --warmup 3 --mode rows --no-cpu-baseline
