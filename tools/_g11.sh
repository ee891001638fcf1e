set -e -o pipefail
O=gpurun_out/pe; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 300 --timeout-method thread > $O/seg_tests.log 2>&1 || { tail -40 $O/seg_tests.log; exit 1; }
tail -1 $O/seg_tests.log
for shape in "--cin 64 --cout 64 --hw 80" "--cin 32 --cout 32 --hw 160"; do
  for env in "VA_PATCH_NW=8" "VA_PATCH_ABL=3"; do
    timeout -k 10 120 python -u tools/conv_micro.py $shape --env $env 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['shape']['batch'],d['shape']['cin'],d['shape']['cout'],d['shape']['hw'],'$env',d['us'],d['tflops'])"
  done
done
timeout -k 10 300 python -u tools/seg_layer_profile.py --batch 64 --iters 10 --json $O/layers.json > $O/layers.log 2>&1
tail -1 $O/layers.log
