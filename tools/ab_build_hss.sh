#!/bin/bash
# Engine variant with extra compiler flags for the Straus kernel's translation unit (cv_k_hss.hip) only,
# into ab/NAME/libcv.so, reusing the other objects of the current in-tree build:
#   tools/ab_build_hss.sh NAME "-mllvm -amdgpu-use-amdgpu-trackers=1"
set -e
NAME=$1; HSSFLAGS=$2
D=ab/$NAME
rm -rf $D && mkdir -p $D/obj
cp corda_amd/_obj/*.o $D/obj/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-ilp $HSSFLAGS \
    -c corda_amd/csrc/cv_k_hss.hip -o $D/obj/cv_k_hss.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libcv.so $D/obj/*.o -lpthread
echo $D/libcv.so
