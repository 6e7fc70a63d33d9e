#!/bin/bash
# Build profiling variants of libmosaic_gpu.so: tools/variants.sh NAME "-DFOO=1" [NAME "-D..."]...
# Each lands in build/ab/NAME/libmosaic_gpu.so (select with MOSAIC_AMD_LIB).  The
# variants' kernels.hip compiles run in parallel; the host objects are the tree's.
set -e
cd "$(dirname "$0")/../mosaic_amd/csrc"
make -s
CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-result -Wno-unused-value"
pids=()
names=()
while [ $# -ge 2 ]; do
  d=../../build/ab/$1; mkdir -p $d
  if [ "${2#all:}" != "$2" ]; then  # NAME "all:-D..." rebuilds both kernels.hip and capi.cpp with the flags
    (/opt/rocm/bin/hipcc $CXXFLAGS ${2#all:} -c capi.cpp -o $d/capi.o 2> $d/build.log &&
     /opt/rocm/bin/hipcc --offload-arch=gfx950 $CXXFLAGS ${2#all:} -c kernels.hip -o $d/kernels.o 2>> $d/build.log &&
     /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libmosaic_gpu.so $d/kernels.o $d/capi.o comm.o tessellate.o \
       bng_format.o h3_glibc.o ring_join.o geom_kernels.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && rm -f $d/capi.o $d/kernels.o) &
  elif [ "${2#host:}" != "$2" ]; then  # NAME "host:-D..." rebuilds capi.cpp (the chip-table builder) instead
    (/opt/rocm/bin/hipcc $CXXFLAGS ${2#host:} -c capi.cpp -o $d/capi.o 2> $d/build.log &&
     /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libmosaic_gpu.so kernels.o $d/capi.o comm.o tessellate.o \
       bng_format.o h3_glibc.o ring_join.o geom_kernels.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && rm -f $d/capi.o) &
  else
  (/opt/rocm/bin/hipcc --offload-arch=gfx950 $CXXFLAGS $2 -c kernels.hip -o $d/kernels.o 2> $d/build.log &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libmosaic_gpu.so $d/kernels.o capi.o comm.o tessellate.o \
     bng_format.o h3_glibc.o ring_join.o geom_kernels.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && rm -f $d/kernels.o) &
  fi
  pids+=($!); names+=($1)
  shift 2
done
for i in "${!pids[@]}"; do wait ${pids[$i]} || { echo "variant ${names[$i]} failed"; exit 1; }; done
