# batch-1 f32 s-seg forward (the drop-in's network) with the split-K layers on conv2 (VA_F32_SMALL=0) or on the
# three-plane kernels (1: stride-1 3x3 on conv3h, 2: every eligible layer); interleaved processes
export TMPDIR=/tmp; mkdir -p gpurun_out/small
for r in 1 2; do for v in 0 1 2; do
  VA_F32_SMALL=$v timeout -k 10 120 python -u tools/c2_prof.py --seg-only --scale s --dtype f32 --iters 300 > gpurun_out/small/v${v}_r${r}.log 2>&1 || exit 1
  echo "v=$v r=$r $(tail -1 gpurun_out/small/v${v}_r${r}.log)"
done; done
