export TMPDIR=/tmp
mkdir -p gpurun_out/xr
L=$PWD/vision_assist_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg.py -k "split_k or conv3t_split" > gpurun_out/xr/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/splitk_sweep.py --settings default --rounds 4 > gpurun_out/xr/new_$r.log 2>&1 || exit $?
  VA355_LIB=$L/libva355_prev.so timeout -k 10 200 python -u tools/splitk_sweep.py --settings default --rounds 4 > gpurun_out/xr/prev_$r.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/xr/new_*.log gpurun_out/xr/prev_*.log > gpurun_out/xr/summary.txt
