# round 4, session c (short): the new tests + parity, the d = 0 A/B, a bench line
bash tools/gpu_step.sh r04_c --testsel "tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_tailwave.py" --ab "--libs build/ab/base.so build/ab/tw1.so build/ab/scan.so build/ab/padall.so build/ab/scan.so:1=60 build/ab/scan.so:1=90 --d 0 --rounds 8" --bench
