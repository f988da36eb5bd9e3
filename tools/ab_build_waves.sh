#!/bin/bash
# Engine variant whose throughput Straus kernel is built for WAVES waves per SIMD (its launch bounds): both the
# kernel's translation unit and the launchers are rebuilt with -DCV_HSS_WAVES=WAVES, into ab/NAME/libcv.so, the
# other objects reused from the current in-tree build.     tools/ab_build_waves.sh NAME WAVES
set -e
NAME=$1; W=$2
D=ab/$NAME
rm -rf $D && mkdir -p $D/obj
cp corda_amd/_obj/*.o $D/obj/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-ilp -DCV_HSS_WAVES=$W \
    -c corda_amd/csrc/cv_k_hss.hip -o $D/obj/cv_k_hss.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-ilp -DCV_HSS_WAVES=$W \
    -c corda_amd/csrc/cv_kernels.hip -o $D/obj/cv_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libcv.so $D/obj/*.o -lpthread \
    -Wl,--version-script=corda_amd/csrc/cordaverify.map
echo $D/libcv.so
