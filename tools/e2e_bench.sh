#!/bin/bash
# End-to-end rate of the drop-in class through its rings (build/bin/r2iq_harness in
# discard mode): producer thread -> input ring -> fft_mt_r2iq worker -> GPU -> output
# ring -> consumer.  Prints the harness lines for d = 0, 1, 4.  Arg: output dir.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${1:-$R/gpurun_out/e2e}; mkdir -p $O
python3 -c "
import sys; sys.path.insert(0, '$R')
from extio_sddc_amd.synth import make_stream
make_stream(64, 'mix')[4096:].tofile('$O/in64.bin')" || exit $?
for d in 0 1 4; do
  timeout -k 10 120 $R/build/bin/r2iq_harness $O/in64.bin 4096 $d 1024 0 0 1.0 - >> $O/e2e.txt 2>&1 || exit $?
done
cat $O/e2e.txt
