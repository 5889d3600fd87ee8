#!/bin/bash
# Build an experiment variant of libmgx with extra -D flags on the stencil
# kernel sources (kernels.hip, wsmooth.hip, xsmooth.hip):
#   tools/build_variant.sh NAME -DFOO=1 ...  -> hpcclassmultigridproject_amd/libmgx_NAME.so
# (load it with MGX_LIB=...; the default build is untouched)
set -e
NAME=$1; shift
D=hpcclassmultigridproject_amd/csrc
make -s -C $D >/dev/null
mkdir -p $D/build/var_$NAME
for f in kernels wsmooth xsmooth; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
      -Wall -Wno-unused-function -Wno-pass-failed "$@" -c -o $D/build/var_$NAME/$f.o $D/$f.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined \
    -o hpcclassmultigridproject_amd/libmgx_$NAME.so \
    $D/build/var_$NAME/kernels.o $D/build/var_$NAME/wsmooth.o $D/build/var_$NAME/xsmooth.o \
    $D/build/mgx.o $D/build/dist.o $D/build/build_id.o -L/opt/rocm/lib -lamdhip64 -lrccl \
    -lpthread -Wl,-rpath,/opt/rocm/lib
echo built hpcclassmultigridproject_amd/libmgx_$NAME.so
