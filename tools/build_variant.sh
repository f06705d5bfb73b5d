#!/bin/bash
# Build a variant of libsddc_ddc.so (the product library) with extra flags for its kernels into
# build/ab/NAME.so, for interleaved A/B timing with tools/ab_libs.py.
# usage: tools/build_variant.sh NAME "extra hipcc flags" [-DMACRO=...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXTRA=$2
O=$R/build/ab/$NAME; mkdir -p $O
C=$R/extio_sddc_amd/csrc
F="-O3 -std=c++17 -fPIC -fno-slp-vectorize -I$C -I$R/include"
hipcc --offload-arch=gfx950 $F $EXTRA -c $C/ddc_persistent.hip -o $O/p.o
hipcc --offload-arch=gfx950 $F $EXTRA -c $C/ddc_channels.hip -o $O/c.o
hipcc --offload-arch=gfx950 $F -c $C/fft_batch.hip -o $O/b.o
hipcc $F -ffp-contract=off -c $C/ddc_runtime.cpp -o $O/r.o
hipcc $F -ffp-contract=off -c $C/filterbank.cpp -o $O/f.o
hipcc $F -ffp-contract=off -c $C/fine_tune.cpp -o $O/n.o
g++ -O3 -std=c++17 -fPIC -mavx2 -mfma -ffp-contract=off -c $C/cpu/fft_avx2.cpp -o $O/c1.o
g++ -O3 -std=c++17 -fPIC -mavx2 -mfma -ffp-contract=off -c $C/cpu/r2iq_cpu.cpp -o $O/c2.o
hipcc --offload-arch=gfx950 -shared $O/p.o $O/c.o $O/b.o $O/r.o $O/f.o $O/n.o $O/c1.o $O/c2.o -o $R/build/ab/$NAME.so -ldl
echo built $R/build/ab/$NAME.so
