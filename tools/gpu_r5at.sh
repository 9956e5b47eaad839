#!/bin/bash
# (1) training step profile + PMC traffic at HEAD (gpu_r5ar.sh); (2) rehearsal of the 2-rank bench
# path on the box's one GPU (ranks share it over gloo: plumbing only, not a measurement)
bash tools/gpu_r5ar.sh ${1:-unknown} || exit $?
OUT=gpurun_out/r5at
mkdir -p $OUT
POSU_SHARED_GPU_REHEARSAL=1 timeout -k 10 700 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/rehearsal2.json 2> $OUT/rehearsal2.err
rc=$?; tail -c 1500 $OUT/rehearsal2.json; tail -5 $OUT/rehearsal2.err; exit $rc
