#!/bin/bash
# Build a variant of libsddc_ddc.so with extra flags for the persistent, channels and wave kernels into build/ab/NAME.so
# usage: tools/build_variant.sh NAME "extra hipcc flags" [-DMACRO=...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXTRA=$2
O=$R/build/ab/$NAME; mkdir -p $O
C=$R/extio_sddc_amd/csrc
F="-O3 -std=c++17 -fPIC -fno-slp-vectorize -I$C -I$R/include"
hipcc --offload-arch=gfx950 $F -c $C/ddc_kernels.hip -o $O/k.o
hipcc --offload-arch=gfx950 $F $EXTRA -c $C/ddc_persistent.hip -o $O/p.o
hipcc --offload-arch=gfx950 $F $EXTRA -c $C/ddc_channels.hip -o $O/c.o
hipcc --offload-arch=gfx950 $F $EXTRA -c $C/ddc_wave.hip -o $O/w.o
hipcc --offload-arch=gfx950 $F -c $C/fft_batch.hip -o $O/b.o
hipcc $F -ffp-contract=off -c $C/ddc_runtime.cpp -o $O/r.o
hipcc $F -ffp-contract=off -c $C/filterbank.cpp -o $O/f.o
hipcc $F -ffp-contract=off -c $C/fine_tune.cpp -o $O/n.o
hipcc --offload-arch=gfx950 -shared $O/k.o $O/p.o $O/c.o $O/w.o $O/b.o $O/r.o $O/f.o $O/n.o -o $R/build/ab/$NAME.so
echo built $R/build/ab/$NAME.so
