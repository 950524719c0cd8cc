cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or engine or graph" > gpurun_out/fused_tests.log 2>&1
step timeout -k 10 400 python bench.py --steps 24 --warmup 3 > gpurun_out/bench_fused.log 2>&1
BFLY_FUSED_DECODE_ROPE=0 step timeout -k 10 400 python bench.py --steps 24 --warmup 3 > gpurun_out/bench_unfused.log 2>&1
