set -o pipefail
mkdir -p gpurun_out
T="1568,224,16,16 400,240,16,16 1632,1568,16,16"
HRT_LIB=ab/libhrt_r03t.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_r03t cornell 2048 2048 10000 $T > gpurun_out/hunt_r03t.log 2>&1 && \
HRT_LIB=ab/libhrt_nofma.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_nofma cornell 2048 2048 10000 $T > gpurun_out/hunt_nofma.log 2>&1 && \
timeout -k 10 300 python -u scripts/box_hunt.py hunt_cur cornell 2048 2048 10000 $T > gpurun_out/hunt_cur.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_custom_scenes.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/custom_tests.log 2>&1
