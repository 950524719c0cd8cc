# Custom all-reduce (IPC) and sharded-layout GPU tests after the self-test / load-batching changes.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest tests/test_custom_ar_gpu.py tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/car_dist_tests.log 2>&1
