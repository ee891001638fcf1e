set -e -o pipefail
O=gpurun_out/wp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > $O/seg_tests.log 2>&1 || { tail -40 $O/seg_tests.log; exit 1; }
tail -1 $O/seg_tests.log
for shape in "--cin 128 --cout 224 --hw 80" "--cin 128 --cout 128 --hw 40" "--cin 256 --cout 256 --hw 20"; do
  for env in "VA_CONV_WP=0" "VA_CONV_WP=1"; do
    timeout -k 10 120 python -u tools/conv_micro.py $shape --env $env 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['shape']['batch'],d['shape']['cin'],d['shape']['cout'],d['shape']['hw'],'$env',d['us'],d['tflops'])"
  done
done
timeout -k 10 300 python -u tools/seg_layer_profile.py --batch 64 --iters 10 --ab VA_CONV_WP > $O/ab.log 2>&1
tail -1 $O/ab.log
