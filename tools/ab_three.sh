#!/bin/bash
# A/B/C of three builds on one box, alternating processes: tools/ab_three.sh LIB_A LIB_B LIB_C [ROUNDS]
set -o pipefail
R=${4:-3}
for i in $(seq $R); do
  for L in "$1" "$2" "$3"; do
    CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag "$L" || exit 1
  done
done
