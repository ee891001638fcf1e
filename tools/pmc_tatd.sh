#!/bin/bash
# Per-layer TA / TD / TCP / TCC / LDS counters of the f32 s-seg forward (B = 64), one rocprofv3 pass per block set.
export TMPDIR=/tmp
O=r3s8
mkdir -p gpurun_out/$O
run() {  # name counters...
  n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/$O/$n -o run -- \
      python3 tools/pmc_forward.py --dtype f32 --batch 64 --out gpurun_out/$O/plan > gpurun_out/$O/$n.log 2>&1
  echo "$n rc=$?"
}
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE && \
run tcp TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE && \
run tcc TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE
