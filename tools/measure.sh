#!/bin/bash
# One GPU measurement pass (run via gpurun): headline bench, alternate workloads,
# rocprofv3 kernel-trace stats, and FETCH_SIZE / WRITE_SIZE PMC passes.
# Usage: bash tools/measure.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo "bench: $(cat $OUT/bench.json | head -c 300)"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --vae none > $OUT/bench_dit.json 2> $OUT/bench_dit.err || exit 1
# (stream2-cfg, stream2-int8 and stream2-vl-per-frame ride in bench.json's "secondary")
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload cfg4 > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --no-probe > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary --no-probe > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 1
echo done
