# round 4, session o: end to end through RadioHandler (benchmark_test procedure) with host chunks
# of 32 (current), 8 and 4 blocks; plus pruned forward pass 2 at d = 4 and FS weights
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r04_o; mkdir -p $O
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur9.so build/ab/grp4.so --d 4 5 6 --rounds 6 > $O/ab_grp4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --libs build/ab/cur9.so build/ab/fsA.so --d 0 --rounds 8 > $O/ab_fsA.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/fs_stamps.py --kernel fs --libs build/ab/c8st1.so > $O/stamps_fs.log 2>&1 || exit $?
cp extio_sddc_amd/lib/libsddc_ddc.so $O/orig.so
for c in 32 8 4; do
  cp build/ab/hc$c.so extio_sddc_amd/lib/libsddc_ddc.so
  timeout -k 10 400 bash tools/e2e_benchmark_test.sh $O/e2e_hc$c > $O/e2e_hc$c.log 2>&1 || { cp $O/orig.so extio_sddc_amd/lib/libsddc_ddc.so; exit 1; }
done
cp $O/orig.so extio_sddc_amd/lib/libsddc_ddc.so; rm -f $O/orig.so
echo done > $O/DONE
