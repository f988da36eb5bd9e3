#!/bin/bash
# Time one build under several internal knob settings (tools/ab_lib.py, CV_KNOBS / CV_VERIFY_MODE),
# each in its own process:  tools/ab_knobs.sh "KNOBS_1" "KNOBS_2" ...   ("-" = defaults;
# "mode0" = the full-width schedule).
set -o pipefail
for k in "$@"; do
  if [ "$k" = "mode0" ]; then
    CV_VERIFY_MODE=0 timeout -k 10 120 python tools/ab_lib.py --tag "$k" || exit 1
  elif [ "$k" = "-" ]; then
    timeout -k 10 120 python tools/ab_lib.py --tag default || exit 1
  else
    CV_KNOBS="$k" timeout -k 10 120 python tools/ab_lib.py --tag "$k" || exit 1
  fi
done
