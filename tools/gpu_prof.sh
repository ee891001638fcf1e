#!/bin/bash
# Profiling pass for profiles/: rocprofv3 kernel trace of a bench.py configuration, its two HBM PMC passes
# (FETCH_SIZE / WRITE_SIZE, separate runs) and the SQ / GRBM pass per layer of the same network (pmc_forward.py).
# Every step has its own time limit (tools/gpu_steps.sh); PMC passes are bounded too (rocprofv3 error-38 hangs).
#   tools/gpu_prof.sh <outdir under gpurun_out> "<pmc_forward args>" [bench args...]
OUT=$1
FWD=$2
shift 2
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
mkdir -p "gpurun_out/$OUT"
export TMPDIR=/tmp
exec bash tools/gpu_steps.sh \
  300 "$OUT/trace.log" -- rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/$OUT/trace" -o run -- \
      python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --extras none --no-ingest "$@" :: \
  180 "$OUT/fetch.log" -- rocprofv3 --pmc FETCH_SIZE --output-format csv -d "gpurun_out/$OUT/fetch" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --no-ingest --extras none "$@" :: \
  180 "$OUT/write.log" -- rocprofv3 --pmc WRITE_SIZE --output-format csv -d "gpurun_out/$OUT/write" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --no-ingest --extras none "$@" :: \
  150 "$OUT/sq.log" -- rocprofv3 --pmc $SQ --output-format csv -d "gpurun_out/$OUT/sq" -o run -- \
      python3 tools/pmc_forward.py $FWD --out "gpurun_out/$OUT/plan" :: \
  150 "$OUT/fetch_l.log" -- rocprofv3 --pmc FETCH_SIZE --output-format csv -d "gpurun_out/$OUT/fetch_l" -o run -- \
      python3 tools/pmc_forward.py $FWD --out "gpurun_out/$OUT/plan" :: \
  150 "$OUT/write_l.log" -- rocprofv3 --pmc WRITE_SIZE --output-format csv -d "gpurun_out/$OUT/write_l" -o run -- \
      python3 tools/pmc_forward.py $FWD --out "gpurun_out/$OUT/plan"
