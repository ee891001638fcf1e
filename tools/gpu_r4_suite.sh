# full GPU suite on the current tree (round 4): one pytest process, per-test time limit, log under gpurun_out/suite
export TMPDIR=/tmp; mkdir -p gpurun_out/suite
timeout -k 10 1100 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread tests > gpurun_out/suite/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/suite/gpu_tests.log
