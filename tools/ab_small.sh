set -o pipefail
for n in 4096 32768; do
  timeout -k 10 120 python tools/ab_lib.py --n $n --msg 32 --rounds 20 --tag "default_n$n" || exit 1
  CV_OPTS=quad_max=0 timeout -k 10 120 python tools/ab_lib.py --n $n --msg 32 --rounds 20 --tag "throughput_n$n" || exit 1
done
