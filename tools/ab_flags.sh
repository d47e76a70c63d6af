#!/bin/bash
# Same-box A/B of whole-model throughput under several bench.py flag sets (interleaved runs):
#   bash tools/ab_flags.sh <rounds> "<flags A>" "<flags B>" ...   (common flags in $AB_BENCH_ARGS)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/ab_flags
for r in $(seq 1 $R); do
  for fl in "$@"; do
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary \
      ${AB_BENCH_ARGS:---vae none} $fl > gpurun_out/ab_flags/out.json 2> gpurun_out/ab_flags/err.txt || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_flags/out.json').read().strip().splitlines()[-1]); print('[$fl]', 'round', $r, 'img/s %.4f' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'attn %.3f' % d['kernels']['attention']['avg_ms'], 'up %.3f' % d['kernels']['mlp_up']['avg_ms'])"
  done
done
