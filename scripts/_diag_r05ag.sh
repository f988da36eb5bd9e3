mkdir -p gpurun_out/r05ag
for L in ab/ws/libcv.so ab/ring/libcv.so; do
  O=c2_sync_only,host,host
  echo "== $L $O"
  CV_LIB_PATH=$L timeout -k 10 400 python -u tools/keyed_context_probe.py --order $O > gpurun_out/r05ag/kc.log 2>&1 || { tail -5 gpurun_out/r05ag/kc.log; exit 1; }
  grep '"step": "host' gpurun_out/r05ag/kc.log | cut -c1-100
done
for R in 1 2; do
for L in ab/scan/libcv.so ab/ring/libcv.so; do
  echo "== notary $L"
  CV_LIB_PATH=$L timeout -k 10 300 python -u tools/notary_probe.py --sizes 16384,32768,65536 --reps 60 --pinned > gpurun_out/r05ag/np.log 2>&1 || { tail -5 gpurun_out/r05ag/np.log; exit 1; }
  grep "^{" gpurun_out/r05ag/np.log | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['n'], 'host', [round(x,3) for x in d['host_p50_p99_ms']], 'pinned', [round(x,3) for x in d['pinned_p50_p99_ms']], d['host_phases_us_mean']['setup'], d['pinned_host_phases_us_mean']['setup'])"
done
done
