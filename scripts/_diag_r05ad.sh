mkdir -p gpurun_out/r05ad
for L in ab/ring/libcv.so ab/prio/libcv.so; do
  for O in c2_sync_only,host host; do
    echo "== $L $O"
    CV_LIB_PATH=$L timeout -k 10 400 python -u tools/keyed_context_probe.py --order $O > gpurun_out/r05ad/kc.log 2>&1 || { tail -5 gpurun_out/r05ad/kc.log; exit 1; }
    grep '"step": "host' gpurun_out/r05ad/kc.log | cut -c1-100
  done
done
