# Prefill-attention kernel variants (BFLY_ATTN_PF_VARIANT: 0 one workgroup per item, 1 round-1 kernel,
# 2 MFMA row sums, 3 persistent item walk = default): correctness, timing table, one PMC pass each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for v in ${TEST_VARIANTS:-3}; do
  BFLY_ATTN_PF_VARIANT=$v step timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn_prefill or lse" > gpurun_out/attn_tests_v$v.log 2>&1
done
step timeout -k 10 300 python tools/bench_attn.py --prefill 16:1024:64:8,4:4096:64:8,1:16384:64:8,64:1024:8:1 --variants ${BENCH_VARIANTS:-0,3} --cases 64:1024:64:8 --kv-dtype bf16 > gpurun_out/attn_variants.log 2>&1
for v in ${PMC_VARIANTS:-3}; do
  BFLY_ATTN_PF_VARIANT=$v step timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_attn_v$v -o run \
    --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU \
    -- python3 tools/bench_attn.py --prefill 16:1024:64:8 --cases 1:256:8:1 --kv-dtype bf16
done
