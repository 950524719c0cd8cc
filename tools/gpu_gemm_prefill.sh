# Prefill-shape GEMMs: our big-tile kernel vs torch.matmul (hipBLASLt) at M = 4096 / 8192 / 16384.
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python tools/bench_gemm.py --ms 4096,8192,16384 --shapes tp1 > gpurun_out/gemm_prefill.log 2>&1
echo "[$?] bench_gemm"
