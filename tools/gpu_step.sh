export TMPDIR=/tmp
mkdir -p gpurun_out/r6f5
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f5/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r6f5/bench.json 2> gpurun_out/r6f5/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f5/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --extras none > gpurun_out/r6f5/rocprof_stats.log 2>&1 || exit $?
