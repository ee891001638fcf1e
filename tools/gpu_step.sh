export TMPDIR=/tmp
mkdir -p gpurun_out/b1h
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b1h/dropin_trace -o run -- python3 bench.py --dropin-only > gpurun_out/b1h/dropin_trace.log 2>&1 || exit $?
timeout -k 10 900 bash tools/ab_c4.sh b1h/c4 2 "VA_SPLITK_OVERLAP=4" "VA_SPLITK_OVERLAP=6" "VA_SPLITK_OVERLAP=12" "VA_SPLITK_OVERLAP=0" > gpurun_out/b1h/ab_c4.log 2>&1 || exit $?
