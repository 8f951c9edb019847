set -o pipefail
mkdir -p gpurun_out
T="1568,224,16,16 400,240,16,16 1632,1568,16,16"
HRT_LIB=ab/libhrt_nofma2.so timeout -k 10 400 python -u scripts/box_hunt.py hunt_nofma2 cornell 2048 2048 10000 $T > gpurun_out/hunt_nofma2.log 2>&1
rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/gpu.sh "tests" "smoke" "bench s3_c2 --steps 5 --no-cpu-baseline --no-delivery" "configs s3" "probe s3_final --preset final --width 800 --height 800 --spp 64 --reps 2 --count" "probe s3_smoke --preset cornell_smoke --width 800 --height 800 --spp 200 --reps 2 --count"
bash scripts/gpu.sh "libs s3_hyb '--preset random_10k --width 3840 --height 2160 --spp 256 --share 8 --reps 3' base anyg" "probe s3_dp_c5 --preset cornell --width 2048 --height 2048 --spp 1250 --share 8 --reps 3 --commit-env HRT_WALK_DP=1/HRT_WALK_DP=0" "probe s3_dp_c2 --preset random --width 1920 --height 1080 --spp 100 --reps 3 --commit-env HRT_WALK_DP=1/HRT_WALK_DP=0"
