# Split-K slab stores: write-through (sc1, default) vs plain write-back, after the C^T epilogue
# rewrite. Kernel tests first (GEMM plans, fused split-K consumers, MoE), then interleaved
# whole-step A/B for Llama-3-70B and Llama-3-8B at B=64 on one GPU.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or moe" > gpurun_out/slab_kernel_tests.log 2>&1
for i in 1 2; do
  step timeout -k 10 300 env BFLY_GEMM_SLAB_WT=1 python bench.py --steps 32 --warmup 4 --out gpurun_out/ab_70b_wt1_$i.json > gpurun_out/ab_70b_wt1_$i.log 2>&1
  step timeout -k 10 300 env BFLY_GEMM_SLAB_WT=0 python bench.py --steps 32 --warmup 4 --out gpurun_out/ab_70b_wt0_$i.json > gpurun_out/ab_70b_wt0_$i.log 2>&1
done
step timeout -k 10 300 env BFLY_GEMM_SLAB_WT=1 python bench.py --model llama3-8b --steps 64 --warmup 4 --out gpurun_out/ab_8b_wt1.json > gpurun_out/ab_8b_wt1.log 2>&1
step timeout -k 10 300 env BFLY_GEMM_SLAB_WT=0 python bench.py --model llama3-8b --steps 64 --warmup 4 --out gpurun_out/ab_8b_wt0.json > gpurun_out/ab_8b_wt0.log 2>&1
grep -h '"ms_per_step"' gpurun_out/ab_*.json | python -c "import sys,json; [print(json.loads(l)['config']['model'], json.loads(l)['ms_per_step'], json.loads(l)['value']) for l in sys.stdin]"
