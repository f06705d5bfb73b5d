#!/bin/bash
# build an existing build/ab/src_NAME tree into build/ab/NAME.so
set -e
R=/root/repo; NAME=$1; S=$R/build/ab/src_$NAME; C=$S/csrc; O=$S/obj; mkdir -p $O
F="-O3 -std=c++17 -fPIC -fno-slp-vectorize -I$C -I$S/include $EXTRA"
objs=""
for k in $C/*.hip; do b=$(basename $k .hip); /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c $k -o $O/$b.o & objs="$objs $O/$b.o"; done
for c in ddc_runtime filterbank fine_tune; do /opt/rocm/bin/hipcc $F -ffp-contract=off -c $C/$c.cpp -o $O/$c.o & objs="$objs $O/$c.o"; done
for c in fft_avx2 r2iq_cpu; do g++ -O3 -std=c++17 -fPIC -mavx2 -mfma -ffp-contract=off -I$C -I$S/include -c $C/cpu/$c.cpp -o $O/cpu_$c.o & objs="$objs $O/cpu_$c.o"; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs -o $R/build/ab/$NAME.so -ldl
echo built $R/build/ab/$NAME.so
