set -e -o pipefail
O=gpurun_out/fk2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > $O/seg_tests.log 2>&1 || { tail -40 $O/seg_tests.log; exit 1; }
tail -1 $O/seg_tests.log
timeout -k 10 120 python -u tools/conv_micro.py --cin 128 --cout 224 --hw 80 --env VA_CONV_WP=0 | tail -1
timeout -k 10 300 python -u tools/seg_layer_profile.py --batch 64 --iters 10 --ab VA_CONV_WP > $O/ab.log 2>&1
tail -1 $O/ab.log
