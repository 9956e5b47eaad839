#!/bin/bash
# r4w: r4u (layer2 chained tail variants) + r4v (layer1 Bottleneck SQ counters)
set -o pipefail
bash tools/gpu_r4u.sh && bash tools/gpu_r4v.sh
