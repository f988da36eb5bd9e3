set -o pipefail
for n in 4096 32768; do
  timeout -k 10 120 python tools/ab_lib.py --n $n --msg 32 --rounds 20 --tag "hsquad_n$n" || exit 1
  CV_KNOBS=cvk_set_hs_quad=0 timeout -k 10 120 python tools/ab_lib.py --n $n --msg 32 --rounds 20 --tag "fullquad_n$n" || exit 1
done
