set -e -o pipefail
O=gpurun_out/abl; mkdir -p $O
for shape in "--cin 128 --cout 224 --hw 80" "--cin 128 --cout 128 --hw 40" "--cin 64 --cout 128 --hw 160 --stride 2"; do
  for env in "VA_CONV3=0" "VA_CONV3=1" "VA_CONV3_ABL=1" "VA_CONV3_ABL=2"; do
    timeout -k 10 120 python -u tools/conv_micro.py $shape --env VA_CONV3_MIN=1 --env $env 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['shape']['cin'],d['shape']['cout'],d['shape']['hw'],'$env',d['us'],d['tflops'])"
  done
done
