export TMPDIR=/tmp
mkdir -p gpurun_out/pmc6
PASSES="sq tcc fetch write" BATCH=256 timeout -k 10 600 bash tools/pmc_conv.sh pmc6/b256 > gpurun_out/pmc6/b256.log 2>&1 || exit $?
PASSES="sq tcc fetch write" BATCH=64 timeout -k 10 400 bash tools/pmc_conv.sh pmc6/b64 > gpurun_out/pmc6/b64.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc6/b1trace -o run -- python3 tools/splitk_sweep.py --scale s --dtype f32 --settings default --rounds 1 --iters 10 > gpurun_out/pmc6/b1trace.log 2>&1 || exit $?
