#!/bin/bash
# A/B timing on one box: alternate two builds of the library (ab/old.so, ab/new.so) through
# bench.py (DH_LIB_PATH), ROUNDS times each, to separate a code change from box-to-box
# clock spread.  Extra bench flags: $BENCH_ARGS.  Output: gpurun_out/ab/{old,new}_<i>.json
set -e
mkdir -p gpurun_out/ab
R=${ROUNDS:-2}
for i in $(seq 1 $R); do
  for v in old new; do
    DH_LIB_PATH=ab/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 $BENCH_ARGS \
      > gpurun_out/ab/${v}_$i.json 2> gpurun_out/ab/${v}_$i.err
    echo "$v $i done"
  done
done
