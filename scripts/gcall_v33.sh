# v33: multi-rank rehearsal of bench.py on the 1-GPU box (2 ranks share the GPU over gloo)
set -o pipefail
O=gpurun_out/v33
mkdir -p $O
export TMPDIR=/tmp
DLSM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-e2e --no-cpu > $O/rehearsal_2ranks.json 2> $O/rehearsal_2ranks.err
