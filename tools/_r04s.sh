# round 4, session s: the schedule-identity tests
set -o pipefail
bash tools/gpu_step.sh r04_s --testsel "tests/test_gpu_queue.py" || exit $?
