#!/bin/bash
# Build a variant of the engine library into ab/NAME/libcv.so from the current sources, with any
# extra files given as SRC=DEST overrides (e.g. /tmp/cv_field_x.h=corda_amd/csrc/cv_field.h).
set -e
NAME=$1; shift
D=ab/$NAME
rm -rf $D && mkdir -p $D/corda_amd/csrc $D/include
cp corda_amd/csrc/*.h corda_amd/csrc/*.hip corda_amd/csrc/*.cpp $D/corda_amd/csrc/
cp include/*.h $D/include/
for o in "$@"; do cp "${o%%=*}" "$D/${o#*=}"; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-ilp -shared $D/corda_amd/csrc/cv_kernels.hip \
    -x hip $D/corda_amd/csrc/cv_api.cpp -o $D/libcv.so -lpthread
echo $D/libcv.so
