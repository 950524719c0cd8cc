# Persistent big prefill GEMM: kernel tests, prefill-shape timing (persistent vs one workgroup per
# tile, BFLY_GEMM_BIG_PERSIST), and the 1-GPU 70B bench.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or moe" > gpurun_out/bigp_tests.log 2>&1
step timeout -k 10 300 env BFLY_GEMM_BIG_PERSIST=0 python tools/bench_gemm.py --ms 4096,8192 --shapes tp1 > gpurun_out/bigp_off.log 2>&1
step timeout -k 10 300 env BFLY_GEMM_BIG_PERSIST=1 python tools/bench_gemm.py --ms 4096,8192 --shapes tp1 > gpurun_out/bigp_on.log 2>&1
step timeout -k 10 400 python bench.py --steps 32 --warmup 4 > gpurun_out/bigp_bench.log 2>&1
