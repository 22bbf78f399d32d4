#!/bin/bash
# Hardware-counter passes (one rocprofv3 --pmc pass each, kernel trace only; no sys/runtime trace) over a
# one-round kbench run. Outputs under gpurun_out/pmc_<tag>_<n>/.
#   tools/pmc_passes.sh <tag> [kbench args...]
set -u
tag=$1; shift
export TMPDIR=/tmp
R=$(pwd)
K="$R/tools/kbench.py --rounds 1 $*"
n=0
while read -r counters; do
    [ -z "$counters" ] && continue
    n=$((n+1))
    tools/gpu_step.sh 600 pmc_${tag}_${n}.log rocprofv3 --pmc $counters -d $R/gpurun_out/pmc_${tag}_${n} -o run --output-format csv -- python3 $K || exit 99
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INST_CYCLES_VMEM_RD
TCC_HIT TCC_MISS GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TA_BUSY_avr
LIST
