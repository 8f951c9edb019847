set -o pipefail
mkdir -p gpurun_out
T="1568,224,16,16 400,240,16,16 1632,1568,16,16"
timeout -k 10 900 python -u -m pytest tests/test_box_forms.py tests/test_custom_scenes.py "tests/test_gpu_configs.py::test_c3_full_frame_exact_equals_reference_traversal" "tests/test_gpu_configs.py::test_c4_share8_exact_equals_reference_traversal" "tests/test_gpu_configs.py::test_c5_share8_exact_equals_reference_traversal" -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s1_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/s1_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu.sh "bench s1_c2 --steps 5 --no-cpu-baseline --no-delivery" "configs s1" "probe s1_final --preset final --width 800 --height 800 --spp 64 --reps 2 --count --commit-env HRT_GWALK_FLATLIST=1/HRT_GWALK_FLATLIST=0" || exit $?
HRT_LIB=ab/libhrt_r03t.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_r03t cornell 2048 2048 10000 $T > gpurun_out/hunt_r03t.log 2>&1 && \
HRT_LIB=ab/libhrt_nofma.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_nofma cornell 2048 2048 10000 $T > gpurun_out/hunt_nofma.log 2>&1
