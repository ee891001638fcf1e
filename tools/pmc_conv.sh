#!/bin/bash
# Per-layer SQ / LDS / TA-TD / TCC counters of the f32 s-seg forward (B = $BATCH, 64 by default; tools/pmc_forward.py),
# one rocprofv3 pass per counter set, each under its own time limit; then tools/pmc_summary.py maps them to layer names.
#   bash tools/pmc_conv.sh OUTDIR [extra env, e.g. VA_CONV3H=0]      (PASSES="sq lds tcc tcp fetch write" by default)
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for kv in "$@"; do export "$kv"; done
PASSES=${PASSES:-sq lds tcc tcp fetch write}
BATCH=${BATCH:-64}
run() {  # name counters...
  n=$1; shift
  case " $PASSES " in *" $n "*) ;; *) return 0;; esac
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- \
      python3 tools/pmc_forward.py --dtype f32 --batch $BATCH --out $O/plan > $O/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; return $rc
}
run sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum TD_TD_BUSY_sum \
    TD_TC_STALL_sum GRBM_GUI_ACTIVE && \
run tcc TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum GRBM_GUI_ACTIVE && \
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
run write WRITE_SIZE GRBM_GUI_ACTIVE && \
python3 tools/pmc_summary.py $O/plan.json $O/summary.json $(for n in $PASSES; do echo $O/$n/*counter_collection.csv; done) \
    > $O/summary.log 2>&1
echo "summary rc=$?"
