set -o pipefail
mkdir -p gpurun_out/g4
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "phased or every_tile or big_tiles or direct or conv" > gpurun_out/g4/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/conv_micro.py --cases deconv3,deconv2,l3c2,l2c2,l1c2,l3c1 --tiles=-1,3,5,29 --rounds 2 --reps 20 --stamps > gpurun_out/g4/micro.txt 2>&1 || exit 2
echo done
