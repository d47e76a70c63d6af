#!/bin/bash
# Bench under torchrun with the collective path on (--force-dist) vs the plain single-process run,
# and the HIP hardware-queue count, to locate the cost of the distributed path at N = 1.
set -o pipefail
mkdir -p gpurun_out/dist
run() {  # name, env, torchrun?, extra args
  local name=$1 envs=$2 tr=$3; shift 3
  if [ "$tr" = 1 ]; then
    env $envs timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --force-dist "$@" \
      > gpurun_out/dist/$name.json 2> gpurun_out/dist/$name.err || return 1
  else
    env $envs timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline "$@" \
      > gpurun_out/dist/$name.json 2> gpurun_out/dist/$name.err || return 1
  fi
  python -c "import json; d=json.loads(open('gpurun_out/dist/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value'], 4), round(d['ms_per_step'], 2))"
}
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
run single "X=1" 0 || exit 1
run dist "X=1" 1 || exit 1
run dist_q8 "GPU_MAX_HW_QUEUES=8" 1 || exit 1
run single_noov "X=1" 0 --no-text-overlap || exit 1
run dist_noov "X=1" 1 --no-text-overlap || exit 1
