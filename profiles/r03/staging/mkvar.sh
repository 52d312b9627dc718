#!/bin/bash
# dev/mkvar.sh NAME "EXTRA FLAGS": libmmadmm.so variant with admm_kernels.hip rebuilt under EXTRA
set -e
cd /root/repo/mm-admm_amd
D=/root/repo/dev/$1; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable $2 -c csrc/kernels/admm_kernels.hip -o $D/admm_kernels.o
OBJS=$(ls build/*.o | grep -v "/admm_kernels.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fopenmp -o $D/libmmadmm.so $D/admm_kernels.o $OBJS -Wl,-rpath,/opt/rocm/lib -lrccl
rm -f $D/admm_kernels.o
