mkdir -p gpurun_out/r05y
O=c2_host_pinned,host
for V in "X=0" "GPU_MAX_HW_QUEUES=8" "HSA_ENABLE_SDMA=0"; do
  echo "== $V"
  env $V timeout -k 10 400 python -u tools/keyed_context_probe.py --order $O > gpurun_out/r05y/kc.log 2>&1 || { tail -5 gpurun_out/r05y/kc.log; exit 1; }
  grep '"step": "host' gpurun_out/r05y/kc.log | cut -c1-110
done
