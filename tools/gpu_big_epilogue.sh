# Big prefill GEMM with the C^T epilogue (8-B bf16 / SiLU stores): kernel tests, prefill-shape timing
# vs hipBLASLt, and the 1-GPU 70B bench (prefill tok/s + decode).
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or moe" > gpurun_out/big_kernel_tests.log 2>&1
step timeout -k 10 500 python tools/bench_gemm.py --ms 8192 --shapes tp1 > gpurun_out/gemm_prefill_ct.log 2>&1
step timeout -k 10 400 python bench.py --steps 32 --warmup 4 > gpurun_out/bench_ct.log 2>&1
