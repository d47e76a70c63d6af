#!/bin/bash
# PMC passes over the standalone attention kernel (tools/ab.py attention, one library):
# stall buckets, LDS bank conflicts and MFMA busy cycles. Usage: bash tools/attn_pmc.sh <out-dir>
set -o pipefail
OUT=${1:-gpurun_out/attn_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=qwen_image_edit_streamdiffusion_amd/libqie.so
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/p1 -o run -- python tools/ab.py attention $LIB@log2q 4 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python tools/ab.py attention $LIB@log2q 4 > $OUT/p2.log 2>&1 || exit 1
echo done
