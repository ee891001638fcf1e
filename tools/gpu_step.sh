export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_w8.py > gpurun_out/t7.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t7.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python -u tools/seg_layer_profile.py --scale m --res 1280 --batch 8 --dtype w8a16 --plan-ab VA_W8 --iters 20 > gpurun_out/l7.log 2>&1
  echo "rc=$?" >> gpurun_out/l7.log
fi
exit $rc
