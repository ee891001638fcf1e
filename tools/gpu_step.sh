export TMPDIR=/tmp
mkdir -p gpurun_out/b1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg.py -k "split_k" > gpurun_out/b1/tests_splitk.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/splitk_sweep.py --scale s --dtype f32 > gpurun_out/b1/sweep_s_f32.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/splitk_sweep.py --scale n --dtype bf16 > gpurun_out/b1/sweep_n_bf16.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/conv2_phases.py --scale s --dtype f32 --batch 1 --reps 5 > gpurun_out/b1/phases_f32_b1_red.log 2>&1 || exit $?
