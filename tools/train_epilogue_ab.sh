# Training-step A/B of the conv epilogue mode (register-direct vs LDS), 8 timed steps each:
#   bash tools/train_epilogue_ab.sh   (on the GPU box, from the repo root)
set -o pipefail
for e in 1 0; do
timeout -k 10 200 python -c "
import sys; sys.argv=['bench.py','--mode','train','--steps','8','--warmup','3']
sys.path[:0]=['pose-unsupervised_amd/lib','.']
from posu import ops
ops.set_conv_epilogue($e)
import bench; bench.main()" 2>&1 | grep metric | cut -c1-220 || exit 1
done
