# round 4, final check of the committed tree (last commit of the round): GPU tests, smoke, the driver's bench command
set -o pipefail
O=gpurun_out/r04_final5; mkdir -p $O
bash tools/gpu_step.sh r04_final5 --tests --bench || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo done > $O/DONE2
