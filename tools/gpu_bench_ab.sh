# 1-GPU bench A/B: default (async decode) vs --sync-decode, plus the CP engine GPU checks.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 400 python bench.py --steps 32 --warmup 4 > gpurun_out/bench_async.log 2>&1
step timeout -k 10 400 python bench.py --steps 32 --warmup 4 --sync-decode > gpurun_out/bench_sync.log 2>&1
step timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread -k "context_parallel" > gpurun_out/cp_tests.log 2>&1
