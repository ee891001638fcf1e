set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc1; mkdir -p $O
timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for v in 0 1; do
  timeout -k 10 120 python -u tools/conv_micro.py --env VA_CONV3=$v --env VA_CONV3_MIN=1 > $O/micro_$v.json 2>&1
  cat $O/micro_$v.json | tail -1
done
for v in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/p1_$v -o run -- python3 tools/conv_micro.py --iters 10 --env VA_CONV3=$v --env VA_CONV3_MIN=1 > $O/p1_$v.log 2>&1
done
echo done
