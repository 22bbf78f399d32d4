#!/bin/bash
# One round's measurement set on the GPU box, everything under gpurun_out/prof_<tag>/:
#   bench.json            the default bench.py line (200 timed steps, CPU baseline included)
#   trace/                rocprofv3 --kernel-trace --stats of a 20-step bench run (kernel_stats.csv)
#   fetch/, write/        one PMC pass each: FETCH_SIZE, WRITE_SIZE (they cannot share a pass)
#   lds/                  LDS counters (bank-conflict and LDS-array cycles, LDS issue stalls) of the full launches
#   l2/                   L2 hits and misses (TCC_HIT_sum, TCC_MISS_sum): the share of the gathers the L2 serves
#   sq/, sq_gram/         SQ counters of the full launches, and of the Gram alone (ALS_DEBUG_SKIP_SOLVE=1, which only
#                         the debug build honours: collaborative-filtering-kafka_amd/build_debug, `make debug`)
# Every GPU step has its own time limit; a fault, abort or timeout ends the script (no further GPU step).
#   tools/profile_round.sh <tag> [extra bench args...]
set -u
tag=$1; shift
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/prof_$tag
mkdir -p "$O"
B="--steps 20 --warmup 2 --no-cpu-baseline $*"
P="--steps 3 --warmup 1 --no-cpu-baseline $*"
KB=$(echo " $* " | grep -o -- "--k [0-9]*" || true)   # kbench takes the bench's --k
ONLY=${ONLY:-}   # ONLY="sq_gram lds": run just these passes
step() {   # step <seconds> <log> <cmd...>
    local secs=$1 log=$2; shift 2
    if [ -n "$ONLY" ] && ! echo " $ONLY " | grep -q " ${log%.*} "; then return 0; fi
    timeout -k 10 "$secs" "$@" > "$O/$log" 2>&1
    local rc=$?
    echo "$(date +%T) rc=$rc $log" | tee -a "$O/steps.log"
    if [ $rc -ne 0 ]; then tail -n 20 "$O/$log"; exit 99; fi
}
step 300 bench.json python3 bench.py $*
step 300 trace.log rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" $B
step 300 fetch.log rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run --output-format csv -- python3 "$R/bench.py" $P
step 300 write.log rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- python3 "$R/bench.py" $P
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE"
step 300 sq.log rocprofv3 --pmc $SQ -d "$O/sq" -o run --output-format csv -- python3 "$R/bench.py" $P
# the Gram alone: the debug build (bench.py refuses it), driven by kbench over the same blocks and kernels
CFK_ALS_LIB=$R/collaborative-filtering-kafka_amd/build_debug/libcfk_als.so \
    step 300 sq_gram.log rocprofv3 --pmc $SQ -d "$O/sq_gram" -o run --output-format csv -- python3 "$R/tools/kbench.py" \
    --rounds 2 --variants ALS_DEBUG_SKIP_SOLVE=1 $KB
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
step 300 lds.log rocprofv3 --pmc $LDS -d "$O/lds" -o run --output-format csv -- python3 "$R/bench.py" $P
step 300 l2.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$O/l2" -o run --output-format csv -- python3 "$R/bench.py" $P
echo "profile_round $tag done"
