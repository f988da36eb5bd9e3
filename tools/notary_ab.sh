#!/bin/bash
for r in 1 2; do
  for L in ab/base/libcv.so ab/cur/libcv.so; do
    CV_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-sub --no-keyed --steps 3 > gpurun_out/nab.log 2>&1 || exit 1
    python - "$L" <<'PY'
import json,sys
d=json.loads([l for l in open("gpurun_out/nab.log") if l.startswith("{")][-1])
n=d["notary"]; sw={s["batch"]:(round(s["p50_ms"],4), round(s["breakdown_p50_ms"]["transfers_and_host"],4)) for s in d["notary_sweep"]}
print(sys.argv[1], "4096", round(n["p50_ms"],4), round(n["breakdown_p50_ms"]["transfers_and_host"],4), sw)
PY
  done
done
