#!/bin/bash
# Serialised GEMM plan sweep under rocprofv3 -> profiles/gemm_tune_<name>.json (run on the GPU box).
# usage: tools/gemm_tune.sh <name> <bench_gemm args...>
set -e
name=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt_$name -o run -- \
    python3 tools/bench_gemm.py --sweep --serial gpurun_out/gt_${name}_log.jsonl "$@"
python3 tools/gemm_trace_tune.py gpurun_out/gt_$name/run_kernel_trace.csv gpurun_out/gt_${name}_log.jsonl \
    --out gpurun_out/gemm_tune_$name.json
rm -rf gpurun_out/gt_$name   # the raw trace is large; the json summary is what we keep
