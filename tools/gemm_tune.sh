#!/bin/bash
# Serialised GEMM plan sweep under rocprofv3 -> gpurun_out/gemm_tune_<name>.json (run on the GPU box).
# usage: tools/gemm_tune.sh <name> <bench_gemm args...>
# The raw kernel trace is deleted whatever happens (it is large; the json summary is kept).
name=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
trap 'rm -rf gpurun_out/gt_$name' EXIT
timeout -k 10 1000 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt_$name -o run -- \
    python3 tools/bench_gemm.py --sweep --serial gpurun_out/gt_${name}_log.jsonl "$@" || exit $?
python3 tools/gemm_trace_tune.py gpurun_out/gt_$name/run_kernel_trace.csv gpurun_out/gt_${name}_log.jsonl \
    --out gpurun_out/gemm_tune_$name.json
