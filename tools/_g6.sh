set -e -o pipefail
for shape in "--cin 64 --cout 64 --hw 80" "--cin 32 --cout 32 --hw 160"; do
  for env in "VA_CONV_PATCH=0" "VA_PATCH_NW=4" "VA_PATCH_NW=8" "VA_PATCH_ABL=1" "VA_PATCH_ABL=2" "VA_PATCH_ABL=3"; do
    timeout -k 10 120 python -u tools/conv_micro.py $shape --env $env 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['shape']['cin'],d['shape']['cout'],d['shape']['hw'],'$env',d['us'],d['tflops'])"
  done
done
