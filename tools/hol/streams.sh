#!/bin/bash
# One process, N CU-masked streams (4 CUs per XCD each), VALU work: does
# in-process multi-queue dispatch keep 8 slices flat where 8 processes do not?
set -e
B=build/holbench
for q in 4 8; do
  for n in 1 4 5 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 5 30 $B --streams $n --iters 1000 --seconds 2 --tag "q$q-s$n"
  done
done
