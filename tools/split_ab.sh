#!/bin/bash
# Same-box A/B of the text-stream split-K configuration (bench.py --text-splits), DiT only.
#   bash tools/split_ab.sh <rounds> cfg1 cfg2 ...
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/split_ab
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --vae none --text-splits "$cfg" \
      > gpurun_out/split_ab/out.json 2> gpurun_out/split_ab/err.txt || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/split_ab/out.json').read().strip().splitlines()[-1]); print('splits $cfg round $r', 'img/s %.4f' % d['value'], 'ms/step %.2f' % d['ms_per_step'])"
  done
done
