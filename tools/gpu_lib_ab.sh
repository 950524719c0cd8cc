# Same-box A/B of two kernel-library builds (BFLY_KERNEL_LIB): ab_libs/_C_base.so (before the C^T
# GEMM epilogue) vs the current butterfly_amd/_C.so, Llama-3-70B at B=1 and B=16.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  for v in base new; do
    lib=$([ $v = base ] && echo ab_libs/_C_base.so || echo butterfly_amd/_C.so)
    step timeout -k 10 300 env BFLY_KERNEL_LIB=$GRAFT_REPO_ROOT/$lib python bench.py --batch-per-gpu 1 --steps 32 --warmup 4 --out gpurun_out/lab_b1_${v}_$i.json > gpurun_out/lab_b1_${v}_$i.log 2>&1
  done
done
for v in base new; do
  lib=$([ $v = base ] && echo ab_libs/_C_base.so || echo butterfly_amd/_C.so)
  step timeout -k 10 300 env BFLY_KERNEL_LIB=$GRAFT_REPO_ROOT/$lib python bench.py --batch-per-gpu 16 --steps 32 --warmup 4 --out gpurun_out/lab_b16_${v}.json > gpurun_out/lab_b16_${v}.log 2>&1
done
