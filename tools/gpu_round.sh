#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats, per-layer profile and the two
# PMC traffic passes.  Every GPU step has its own time limit; the first failure ends the script.
#   tools/gpu_round.sh <tag> [steps]     (outputs under gpurun_out/<tag>/)
set -e -o pipefail
TAG=${1:-run}
STEPS=${2:-20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ -z "$SKIP_TESTS" ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if [ -z "$SKIP_BENCH" ]; then
step bench
timeout -k 10 400 python -u bench.py --steps "$STEPS" > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
step bench-noprof
timeout -k 10 300 python -u bench.py --steps "$STEPS" --no-prof --cpu-sample 0 > "$OUT/bench_noprof.json" 2> "$OUT/bench_noprof.err"
cat "$OUT/bench_noprof.json"
step layers
timeout -k 10 300 python -u tools/seg_layer_profile.py --batch 64 --iters 10 --json "$OUT/layers.json" > "$OUT/layers.log" 2>&1
tail -1 "$OUT/layers.log"
fi
step rocprof-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --extras none > "$OUT/rocprof_stats.log" 2>&1
if [ -z "$SKIP_PMC" ]; then
  step pmc-fetch
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --no-ingest --extras none > "$OUT/pmc_fetch.log" 2>&1
  step pmc-write
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --no-ingest --extras none > "$OUT/pmc_write.log" 2>&1
fi
step done
