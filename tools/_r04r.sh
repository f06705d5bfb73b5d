# round 4, session r: FS slot weights; the final tree's GPU tests, smoke and bench
set -o pipefail
O=gpurun_out/r04_r; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur11.so build/ab/fsB.so build/ab/fsC.so --d 0 --rounds 10 > $O/ab_fs.log 2>&1 || exit $?
bash tools/gpu_step.sh r04_r --tests --bench || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo done > $O/DONE2
