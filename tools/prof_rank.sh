#!/bin/bash
# rocprofv3 kernel trace of ONE rank of a `python -m butterfly_amd launch` job: the launcher
# (which never touches the GPU) starts this wrapper per rank, and the wrapper starts the
# profiler with the program itself after `--`.
#   python -m butterfly_amd launch -n 4 -- bash tools/prof_rank.sh TAG python3 tools/ep_trace.py ...
# -> gpurun_out/prof_TAG/rank<RANK>/run_kernel_trace.csv
# PROF_ARGS overrides the trace domains (e.g. "--kernel-trace --hip-runtime-trace --marker-trace"
# for tools/sync_audit.py; never counters together with API traces).
tag=$1
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof_$tag/rank${RANK:-0}
mkdir -p "$out"
exec rocprofv3 ${PROF_ARGS:---kernel-trace} --output-format csv -d "$out" -o run -- "$@"
