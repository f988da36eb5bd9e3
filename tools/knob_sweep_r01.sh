set -o pipefail
mkdir -p gpurun_out/knobs
for rep in 1 2; do
for k in "" "cvk_set_hs_waves=2" "cvk_set_split_pct=10" "cvk_set_split_pct=40" "cvk_set_split_mode=0"; do
  CV_KNOBS="$k" timeout -k 10 120 python -u tools/ab_lib.py --tag "r$rep:$k" --rounds 9 2>/dev/null | tail -1 || exit 1
done; done
