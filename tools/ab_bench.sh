#!/bin/bash
# Same-box A/B of whole-model throughput for several builds of libqie.so (interleaved runs):
#   bash tools/ab_bench.sh <rounds> lib1.so lib2.so ...   (extra bench.py flags in $AB_BENCH_ARGS)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/ab_bench
for r in $(seq 1 $R); do
  for lib in "$@"; do
    QIE_LIB_PATH=$(realpath $lib) timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline \
      ${AB_BENCH_ARGS:---vae none} > gpurun_out/ab_bench/out.json 2> gpurun_out/ab_bench/err.txt || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench/out.json').read().strip().splitlines()[-1]); print('$lib', 'round', $r, 'img/s %.4f' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'attn %.3f' % d['kernels']['attention']['avg_ms'])"
  done
done
