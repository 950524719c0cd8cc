#!/bin/bash
# In-situ GEMM plan A/B: bench.py once per BFLY_GEMM_PLAN override (';'-separated overrides per
# variant, "base" = the tuned table), each run under its own time limit; prints ms/step per variant.
#   tools/plan_ab.sh "BENCH_ARGS" base "N,K,M:kind,mt,nt,wk,bm,bn,sk" ...   -> gpurun_out/plan_ab.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
args=$1
shift
for v in "$@"; do
  if [ "$v" = base ]; then unset BFLY_GEMM_PLAN; else export BFLY_GEMM_PLAN="$v"; fi
  timeout -k 10 300 python bench.py $args > gpurun_out/plan_ab_run.log 2>&1 || { echo "[$?] $v" | tee -a gpurun_out/plan_ab.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/plan_ab_run.log)" | tee -a gpurun_out/plan_ab.log
done
