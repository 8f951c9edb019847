set -o pipefail
mkdir -p gpurun_out
T="1568,224,16,16 400,240,16,16 1632,1568,16,16"
HRT_LIB=ab/libhrt_r03t.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_r03t cornell 2048 2048 10000 $T > gpurun_out/hunt_r03t.log 2>&1 && \
HRT_LIB=ab/libhrt_nofma.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_nofma cornell 2048 2048 10000 $T > gpurun_out/hunt_nofma.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/gpu.sh "tests test_c5_share8_exact or test_device_box_test" "profile r04a_c2 random 1920 1080 500" "profile r04a_c3 earth_perlin 1920 1080 1000" "profile r04a_c4s8 random_10k 3840 2160 2000 8" "profile r04a_c5s8 cornell 2048 2048 10000 8"
