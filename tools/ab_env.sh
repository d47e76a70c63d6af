#!/bin/bash
# Same-box A/B of whole-model throughput under several environment settings (interleaved runs):
#   bash tools/ab_env.sh <rounds> "VAR=a" "VAR=b" ...   (extra bench.py flags in $AB_BENCH_ARGS)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/ab_env
for r in $(seq 1 $R); do
  for kv in "$@"; do
    env $kv timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline \
      ${AB_BENCH_ARGS:---vae none} > gpurun_out/ab_env/out.json 2> gpurun_out/ab_env/err.txt || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_env/out.json').read().strip().splitlines()[-1]); print('$kv', 'round', $r, 'img/s %.4f' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'attn %.3f' % d['kernels']['attention']['avg_ms'])"
  done
done
