set -o pipefail
mkdir -p gpurun_out/prio
for r in 1 2; do
  for cfg in "0 qwen_image_edit_streamdiffusion_amd/libqie.so" "-1 qwen_image_edit_streamdiffusion_amd/libqie.so" "0 tools/ab_build/noearly.so"; do
    set -- $cfg
    QIE_SIDE_PRIORITY=$1 QIE_LIB_PATH=$(realpath $2) timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --vae none > gpurun_out/prio/out.json 2> gpurun_out/prio/err.txt || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/prio/out.json').read().strip().splitlines()[-1]); print('prio $1 $2 round $r', 'img/s %.4f' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'attn %.3f' % d['kernels']['attention']['avg_ms'])"
  done
done
