# round 4, session b: GPU tests on the working tree; A/B of the FS trims / padding / static share
# (d = 0) and of the tail-wave kernel / static share (d = 1..4); a bench line; stamps
bash tools/gpu_step.sh r04_b --tests --ab "--libs build/ab/base.so build/ab/tw1.so build/ab/padall.so build/ab/tw1.so:1=60 build/ab/tw1.so:1=90 build/ab/tw1.so:1=0 --d 0 --rounds 8" --bench || exit $?
O=gpurun_out/r04_b
timeout -k 10 600 python -u tools/ab_libs.py --libs build/ab/base.so build/ab/tw1.so build/ab/tw1.so:3=0 build/ab/tw1.so:2=100 build/ab/tw1.so:2=50 --d 1 2 3 4 --rounds 6 > $O/ab_p.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/fs_stamps.py --kernel fs --libs build/ab/stamps1.so build/ab/stamps2.so > $O/stamps_fs.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/fs_stamps.py --kernel p --d 4 --libs build/ab/stamps1.so build/ab/stamps2.so > $O/stamps_p4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/fs_stamps.py --kernel p --d 3 --libs build/ab/stamps1.so build/ab/stamps2.so > $O/stamps_p3.log 2>&1 || exit $?
