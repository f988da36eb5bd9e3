mkdir -p gpurun_out/r05ah
for L in ab/rmin/libcv.so ab/cur/libcv.so; do
  O=c2_sync_only,host,host
  echo "== $L $O"
  CV_LIB_PATH=$L timeout -k 10 400 python -u tools/keyed_context_probe.py --order $O > gpurun_out/r05ah/kc.log 2>&1 || { tail -5 gpurun_out/r05ah/kc.log; exit 1; }
  grep '"step": "host' gpurun_out/r05ah/kc.log | cut -c1-100
done
