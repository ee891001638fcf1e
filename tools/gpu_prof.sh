#!/bin/bash
# Profiling pass for profiles/: rocprofv3 kernel trace of the headline bench, the two HBM PMC passes
# (FETCH_SIZE / WRITE_SIZE, separate runs) and the SQ / GRBM pass per layer for the f32 and bf16 forwards.
# Every step has its own time limit; PMC passes are SIGKILLed if they hang (rocprofv3 error-38 behaviour).
#   tools/gpu_prof.sh <outdir> [bench args...]
OUT=$1
shift
BARGS="$*"
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
exec tools/gpu_steps.sh "$OUT" \
  "300:trace:rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --extras none --no-ingest $BARGS" \
  "180:fetch:rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --extras none $BARGS" \
  "180:write:rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --extras none $BARGS" \
  "120:sq_f32:rocprofv3 --pmc $SQ --output-format csv -d $OUT/sq_f32 -o run -- python3 tools/pmc_forward.py --dtype f32 --out $OUT/plan_f32" \
  "120:sq_bf16:rocprofv3 --pmc $SQ --output-format csv -d $OUT/sq_bf16 -o run -- python3 tools/pmc_forward.py --dtype bf16 --out $OUT/plan_bf16" \
  "120:fetch_f32:rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_f32 -o run -- python3 tools/pmc_forward.py --dtype f32 --out $OUT/plan_f32" \
  "120:write_f32:rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_f32 -o run -- python3 tools/pmc_forward.py --dtype f32 --out $OUT/plan_f32"
