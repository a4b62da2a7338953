timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04ff_rollout.log 2>&1
rc=$?; tail -n 20 gpurun_out/r04ff_rollout.log; exit $rc
