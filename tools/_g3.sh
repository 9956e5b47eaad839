set -o pipefail
mkdir -p gpurun_out/g3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "phased or every_tile or big_tiles" > gpurun_out/g3/tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_micro.py --cases l2c2,l3c2,l3c3,deconv1,deconv2,deconv3 --tiles=5,29 > gpurun_out/g3/micro.txt 2>&1 || exit 2
echo done
