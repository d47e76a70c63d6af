#!/bin/bash
# Effective clock of the attention and big-GEMM kernels under load (MI355X_MICROARCH.md
# "DVFS give-back": clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel time), via gpurun:
#   bash tools/clock_probe.sh <outdir>
set -o pipefail
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
LIB=qwen_image_edit_streamdiffusion_amd/libqie.so
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/attn -o run -- python tools/ab.py attention $LIB@log2q 6 > $OUT/attn.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/up -o run -- python tools/ab.py gemm_up $LIB 6 > $OUT/up.log 2>&1 || exit 1
AB_ZERO=1 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/upz -o run -- python tools/ab.py gemm_up $LIB 6 > $OUT/upz.log 2>&1 || exit 1
AB_ZERO=1 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/attnz -o run -- python tools/ab.py attention $LIB@log2q 6 > $OUT/attnz.log 2>&1 || exit 1
find $OUT -name '*.csv' | head -20
