export TMPDIR=/tmp
mkdir -p gpurun_out/w3t
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/w3t/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --no-ingest --extras none > gpurun_out/w3t/fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/w3t/write -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-prof --no-ingest --extras none > gpurun_out/w3t/write.log 2>&1 || exit $?
PASSES="fetch write" BATCH=256 timeout -k 10 400 bash tools/pmc_conv.sh w3t/b256 > gpurun_out/w3t/b256.log 2>&1 || exit $?
