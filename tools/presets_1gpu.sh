#!/bin/bash
# Measure every BASELINE.json config that fits one MI355X (the 8-GPU TP/EP
# layouts are run at TP=1/EP=1 here; 70B bf16 = 141 GB fits in 288 GB HBM).
# Each run has its own time limit; stop at the first fault/timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out/presets
run() {
  name=$1; shift
  echo "== $name: $*"
  timeout -k 10 420 python bench.py "$@" > gpurun_out/presets/$name.log 2>&1
  e=$?
  grep '^{"metric"' gpurun_out/presets/$name.log | tail -1
  echo "== exit $e"
  case $e in 0) ;; *) tail -5 gpurun_out/presets/$name.log; exit $e;; esac
}
for p in "$@"; do
  case $p in
    # the driver's step contract (--steps 20 --warmup 5: 16 completed analyses per step)
    8b-1k)     run 8b-1k --preset llama3-8b-1k --steps 20 --warmup 5 --no-hints-steps 0 ;;
    8b-100k)   run 8b-100k --preset llama3-8b-100k --steps 20 --warmup 5 --no-hints-steps 0 ;;
    mixtral)   run mixtral --preset mixtral-10k --steps 10 --warmup 3 --no-hints-steps 0 ;;
    70b-tp1)   run 70b-tp1 --preset llama3-70b-tp8-10k --tp 1 --incidents 32 --quantum 4 --steps 5 --warmup 2 \
                   --no-hints-steps 0 ;;
    8b-192)    run 8b-192 --incidents 192 --steps 20 --warmup 5 --no-hints-steps 0 ;;
  esac
done
