# Same-box A/B of the headline: this tree against ab_old/ (a copy of the previous commit's Python package, bench.py,
# workloads/ and its libva355.so built with tools/build_variant.sh; not committed), then the FETCH / WRITE passes at B = 256.
set -o pipefail
mkdir -p gpurun_out/w3g
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --extras none --cpu-sample 0 --no-ingest > gpurun_out/w3g/new_$r.json 2> gpurun_out/w3g/new_$r.err || exit 1
  (cd ab_old && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --extras none --cpu-sample 0 --no-ingest) > gpurun_out/w3g/old_$r.json 2> gpurun_out/w3g/old_$r.err || exit 1
done
for f in gpurun_out/w3g/*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['roofline']['achieved'],d['roofline']['frac'])"; done
PASSES="fetch write" BATCH=256 timeout -k 10 400 bash tools/pmc_conv.sh w3g/b256 > gpurun_out/w3g/pmc.log 2>&1 || exit 1
python3 tools/pmc_traffic.py traffic gpurun_out/w3g/b256/fetch/run_counter_collection.csv gpurun_out/w3g/b256/write/run_counter_collection.csv s-640-b256-f32 gpurun_out/w3g/conv_traffic.json
