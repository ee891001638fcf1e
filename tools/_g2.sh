set -e -o pipefail
mkdir -p gpurun_out/c3
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c3/seg_tests.log 2>&1 || { tail -30 gpurun_out/c3/seg_tests.log; exit 1; }
tail -3 gpurun_out/c3/seg_tests.log
timeout -k 10 300 python -u tools/seg_layer_profile.py --batch 64 --iters 10 --ab VA_CONV3 --env VA_CONV3_MIN=1 > gpurun_out/c3/ab_min1.log 2>&1
tail -1 gpurun_out/c3/ab_min1.log
timeout -k 10 300 python -u bench.py --steps 20 --cpu-sample 0 > gpurun_out/c3/bench.json 2>gpurun_out/c3/bench.err
cat gpurun_out/c3/bench.json
timeout -k 10 300 python -u bench.py --steps 20 --cpu-sample 0 --no-prof > gpurun_out/c3/bench_noprof.json 2>>gpurun_out/c3/bench.err
cat gpurun_out/c3/bench_noprof.json
