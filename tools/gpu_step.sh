export TMPDIR=/tmp
L=$PWD/vision_assist_amd
timeout -k 10 1000 bash tools/ab_headline.sh ab6/libs 2 "VA355_LIB=$L/libva355_nodead.so" "VA355_LIB=$L/libva355_c2cb.so" "VA355_LIB=$L/libva355_r5.so" > gpurun_out/ab6_libs.log 2>&1 || exit $?
