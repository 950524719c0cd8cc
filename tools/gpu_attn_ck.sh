# Persistent prefill attention with key chunks (cu_k) and the context-parallel GPU tests.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or lse" > gpurun_out/attn_ck_tests.log 2>&1
step timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/attn_ck_dist.log 2>&1
