#!/bin/bash
# Same-box A/B of whole-model throughput across library builds and bench.py flag sets (interleaved):
#   bash tools/ab_libs.sh <rounds> "<lib.so or -> <flags>" ...   ("-" = the in-tree libqie.so)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/ab_flags
for r in $(seq 1 $R); do
  for spec in "$@"; do
    lib=${spec%% *}; fl=${spec#* }; [ "$fl" = "$spec" ] && fl=""
    if [ "$lib" = "-" ]; then unset QIE_LIB_PATH; else export QIE_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary \
      ${AB_BENCH_ARGS:---vae none} $fl > gpurun_out/ab_flags/out.json 2> gpurun_out/ab_flags/err.txt || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_flags/out.json').read().strip().splitlines()[-1]); print('[$spec]', 'round', $r, 'img/s %.4f' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'attn %.3f' % d['kernels']['attention']['avg_ms'], 'up %.3f' % d['kernels']['mlp_up']['avg_ms'])"
  done
done
