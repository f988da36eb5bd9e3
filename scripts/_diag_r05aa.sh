mkdir -p gpurun_out/r05aa
export TMPDIR=/tmp
for O in host c2_host_pinned,host; do
  echo "== $O"
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r05aa/tl_$O -o tl --output-format csv -- \
     python3 -u tools/keyed_context_probe.py --order $O --calls 4 > gpurun_out/r05aa/kc_$O.log 2>&1 || { tail -5 gpurun_out/r05aa/kc_$O.log; exit 1; }
  grep '"step": "host' gpurun_out/r05aa/kc_$O.log | cut -c1-100
  TL_GAP_MS=3 python3 tools/host_timeline.py --summarize gpurun_out/r05aa/tl_$O > gpurun_out/r05aa/sum_$O.txt 2>&1
  tail -1 gpurun_out/r05aa/sum_$O.txt
  find gpurun_out/r05aa/tl_$O -name "*.csv" -size +20M -delete
done
