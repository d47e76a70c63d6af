#!/bin/bash
# PMC passes for the attention kernel of one libqie build (run via gpurun):
#   bash tools/pmc_attention.sh <lib.so> <outdir>
# Two passes (8 SQ counters each), kernel-trace off; the library is copied in place first.
set -o pipefail
LIB=$1; OUT=$2
mkdir -p $OUT
export TMPDIR=/tmp
cp $LIB qwen_image_edit_streamdiffusion_amd/libqie.so || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -o run -- python tools/kbench.py one attention > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o run -- python tools/kbench.py one attention > $OUT/p2.log 2>&1 || exit 1
