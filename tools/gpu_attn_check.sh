# Prefill-attention correctness + timing, then the CP / SP sharded-layout checks (one GPU).
# A step that crashes, faults or times out ends the script (rc other than 0/1).
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "attn_prefill or lse" -o log_cli=false > gpurun_out/attn_tests.log 2>&1
step timeout -k 10 120 python tools/bench_attn.py --prefill 16:1024:64:8,4:4096:64:8,1:16384:64:8,64:1024:8:1 --cases 64:1024:64:8 --kv-dtype bf16 > gpurun_out/attn_bench.log 2>&1
step timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread -k "context_parallel or sharded_layout" > gpurun_out/dist_tests.log 2>&1
