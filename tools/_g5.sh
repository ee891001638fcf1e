set -e -o pipefail
O=gpurun_out/patch; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -v --timeout 300 --timeout-method thread > $O/seg_tests.log 2>&1 || { tail -40 $O/seg_tests.log; exit 1; }
tail -3 $O/seg_tests.log
timeout -k 10 300 python -u tools/seg_layer_profile.py --batch 64 --iters 10 --ab VA_CONV_PATCH > $O/ab.log 2>&1
tail -1 $O/ab.log
timeout -k 10 300 python -u bench.py --steps 20 --cpu-sample 0 > $O/bench.json 2>$O/bench.err
cat $O/bench.json
