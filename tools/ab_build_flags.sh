#!/bin/bash
# Build a variant of the engine library into ab/NAME/libcv.so from the current sources with extra
# compiler flags for the throughput kernels' translation unit (cv_k_hs.hip) only:
#   tools/ab_build_flags.sh NAME "-mllvm -amdgpu-use-amdgpu-trackers=1"
set -e
NAME=$1; HSFLAGS=$2
D=ab/$NAME
rm -rf $D && mkdir -p $D/obj
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-ilp"
cp corda_amd/_obj/*.o $D/obj/
/opt/rocm/bin/hipcc $F $HSFLAGS -c corda_amd/csrc/cv_k_hs.hip -o $D/obj/cv_k_hs.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libcv.so $D/obj/*.o -lpthread
echo $D/libcv.so
