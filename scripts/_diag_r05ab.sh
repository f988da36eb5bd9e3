mkdir -p gpurun_out/r05ab
for L in ab/eager/libcv.so corda_amd/libcordaverify.so; do
  echo "== $L"
  CV_LIB_PATH=$L timeout -k 10 400 python -u tools/keyed_context_probe.py --order c2_host_pinned,host > gpurun_out/r05ab/kc.log 2>&1 || { tail -5 gpurun_out/r05ab/kc.log; exit 1; }
  grep '"step": "host' gpurun_out/r05ab/kc.log | cut -c1-100
done
