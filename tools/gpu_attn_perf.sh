# Prefill-attention correctness (long / varlen / LSE vs fp32) then timing. Stops on a crash.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn_prefill or lse" > gpurun_out/attn_tests.log 2>&1
step timeout -k 10 120 python tools/bench_attn.py --prefill 16:1024:64:8,4:4096:64:8,1:16384:64:8,64:1024:8:1 --cases 64:1024:64:8 --kv-dtype bf16 > gpurun_out/attn_bench.log 2>&1
