mkdir -p gpurun_out/r05ac
for O in c2_sync_only,host c2_async_only,host; do
  echo "== $O"
  timeout -k 10 400 python -u tools/keyed_context_probe.py --order $O > gpurun_out/r05ac/kc.log 2>&1 || { tail -5 gpurun_out/r05ac/kc.log; exit 1; }
  grep '"step": "host' gpurun_out/r05ac/kc.log | cut -c1-100
done
