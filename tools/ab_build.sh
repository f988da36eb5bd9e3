#!/bin/bash
# Build a variant of the engine library into ab/NAME/libcv.so from the current sources, with any
# extra files given as SRC=DEST overrides (e.g. /tmp/cv_field_x.h=corda_amd/csrc/cv_field.h).
# The kernel translation units compile in parallel (cv_kcommon.h).
set -e
NAME=$1; shift
D=ab/$NAME
rm -rf $D && mkdir -p $D/corda_amd/csrc $D/include $D/obj
cp corda_amd/csrc/*.h corda_amd/csrc/*.hip corda_amd/csrc/*.cpp $D/corda_amd/csrc/
cp include/*.h $D/include/
for o in "$@"; do cp "${o%%=*}" "$D/${o#*=}"; done
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
pids=()
for s in $D/corda_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=max-ilp -c $s -o $D/obj/$(basename $s .hip).o & pids+=($!)
done
/opt/rocm/bin/hipcc -x hip $F -c $D/corda_amd/csrc/cv_api.cpp -o $D/obj/cv_api.o & pids+=($!)
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libcv.so $D/obj/*.o -lpthread
echo $D/libcv.so
