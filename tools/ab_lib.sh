#!/bin/bash
# A/B two builds of the engine on one box, alternating processes: tools/ab_lib.sh LIB_A LIB_B [ROUNDS]
set -o pipefail
A=$1; B=$2; R=${3:-3}
for i in $(seq $R); do
  CV_LIB_PATH=$A timeout -k 10 120 python tools/ab_lib.py --tag A || exit 1
  CV_LIB_PATH=$B timeout -k 10 120 python tools/ab_lib.py --tag B || exit 1
done
