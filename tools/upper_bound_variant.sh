#!/bin/bash
# Timing-only variant of libmgx (WRONG results, never the product): the cross
# pass reads its coarse-u rows from a 32-row window and the zero-input row
# marches read their rhs rows from one -- L2-resident data in place of the
# HBM hand-offs the three-role pass would avoid: its upper bound (DESIGN.md
# section 7b).  Writes hpcclassmultigridproject_amd/libmgx_probe.so; compare
# with MGX_LIB=... python tools/ab_levels.py --fp fma.
set -e
T=/tmp/probe_src; rm -rf $T; mkdir -p $T
cp hpcclassmultigridproject_amd/csrc/*.hip hpcclassmultigridproject_amd/csrc/*.h $T/
sed -i 's|const double \*p0 = uc + rowoff(Rc >> 1, ipc);|const double *p0 = uc + rowoff((Rc >> 1) \& 31, ipc);|' $T/xsmooth.hip
grep -c "(Rc >> 1) & 31" $T/xsmooth.hip
sed -i 's|if (!C::RHSN) d.r = ld2((rhs + o) + cl);|if (!C::RHSN) d.r = ld2((C::ZERO ? rhs + rowoff(Rc \& 31, ip) : rhs + o) + cl);|' $T/wsmooth.hip
grep -c "Rc & 31, ip" $T/wsmooth.hip
D=hpcclassmultigridproject_amd/csrc
for f in kernels wsmooth xsmooth; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
      -Wno-unused-function -Wno-pass-failed -I$D -c -o $T/$f.o $T/$f.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined \
    -o hpcclassmultigridproject_amd/libmgx_probe.so $T/kernels.o $T/wsmooth.o $T/xsmooth.o \
    $D/build/mgx.o $D/build/dist.o $D/build/build_id.o -L/opt/rocm/lib -lamdhip64 -lrccl \
    -lpthread -Wl,-rpath,/opt/rocm/lib
