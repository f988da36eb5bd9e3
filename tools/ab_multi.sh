#!/bin/bash
# A/B/C... several builds of the engine on one box, alternating processes:
#   tools/ab_multi.sh ROUNDS LIB_A LIB_B [LIB_C ...]      (extra ab_lib.py args via AB_ARGS)
set -o pipefail
R=$1; shift
for i in $(seq $R); do
  for L in "$@"; do
    CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag $L $AB_ARGS || exit 1
  done
done
