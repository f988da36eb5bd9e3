mkdir -p gpurun_out/r05x
for O in c2_host_other_engine,host c2_host_pinned,host,host; do
  echo "== $O"
  timeout -k 10 400 python -u tools/keyed_context_probe.py --order $O > gpurun_out/r05x/kc_$O.log 2>&1 || { tail -5 gpurun_out/r05x/kc_$O.log; exit 1; }
  grep '"step": "host' gpurun_out/r05x/kc_$O.log | cut -c1-120
done
