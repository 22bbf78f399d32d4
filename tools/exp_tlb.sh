# address-path counters of the k = 64 launches (TA / TD / TCP incl. UTCL1 translation), one pass each
set -u
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/prof_tlb; mkdir -p $O
P="--steps 3 --warmup 1 --no-cpu-baseline $*"
pass() {
    local n=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$n" -o run --output-format csv -- python3 "$R/bench.py" $P > $O/$n.log 2>&1
    local rc=$?; echo "pass $n rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$n.log; exit 99; }; return 0
}
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
pass utcl1 TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
pass tcp TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE
echo "exp_tlb done"
