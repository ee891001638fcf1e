export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 400 python -u bench.py --scale m --res 1280 --dtype fp8 --regime dense_box --steps 20 --warmup 3 --extras none --cpu-sample 0 --no-ingest > gpurun_out/c5/w8a8_fresh.json 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --scale m --res 1280 --dtype w8a16 --regime dense_box --steps 20 --warmup 3 --extras c5_w8a8 --cpu-sample 0 --no-ingest > gpurun_out/c5/w8a16_then_w8a8.json 2>&1 || exit $?
bash tools/gpu_prof.sh c5/prof "--scale m --res 1280 --batch 8 --dtype w8a16" --scale m --res 1280 --dtype w8a16 --regime dense_box
