mkdir -p gpurun_out/r05z
O=host,dma1,host,dma1,host,dma1,host,dma1,host
timeout -k 10 400 python -u tools/keyed_context_probe.py --calls 6 --order $O > gpurun_out/r05z/kc.log 2>&1 || { tail -5 gpurun_out/r05z/kc.log; exit 1; }
grep '"step": "host' gpurun_out/r05z/kc.log | cut -c1-80
O=c2_host_pinned,host,dma1,host,dma1,host,dma1,host
timeout -k 10 400 python -u tools/keyed_context_probe.py --calls 6 --order $O > gpurun_out/r05z/kc2.log 2>&1 || { tail -5 gpurun_out/r05z/kc2.log; exit 1; }
grep '"step": "host' gpurun_out/r05z/kc2.log | cut -c1-80
