#!/bin/bash
# (1) warm vs cold-cache tile timings on the layer4 / deconv1 shapes (is the in-graph slowdown of
# layer4 against tools/tile_micro.py cache state?); (2) the training step's HBM traffic at HEAD
# (separate FETCH_SIZE / WRITE_SIZE passes, reduced beside posu.roofline's training classes)
OUT=gpurun_out/r5u
COMMIT=${1:-unknown}
mkdir -p $OUT
export TMPDIR=/tmp
T="--tiles 20,4,15,39,23,3 --only l4,deconv1 --reps 10 --rounds 3"
timeout -k 10 200 python -u tools/tile_micro.py $T > $OUT/tile_warm.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/tile_micro.py $T --flush > $OUT/tile_cold.txt 2>&1 || exit $?
echo tiles done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/tf" -o run -- \
  python3 bench.py --mode train --steps 2 --warmup 1 > "$OUT/tf.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/tw" -o run -- \
  python3 bench.py --mode train --steps 2 --warmup 1 > "$OUT/tw.log" 2>&1 || exit $?
POSU_COMMIT=$COMMIT python3 tools/pmc_train_traffic.py "$OUT"/tf/run_counter_collection.csv \
  "$OUT"/tw/run_counter_collection.csv > "$OUT/pmc_traffic_train.txt"
rm -f "$OUT"/tf/*.csv "$OUT"/tw/*.csv
cat $OUT/tile_warm.txt $OUT/tile_cold.txt $OUT/pmc_traffic_train.txt
