#!/bin/bash
# rocprofv3 kernel trace of a short decode benchmark; summary CSVs land in gpurun_out/prof_<tag>.
# usage: tools/profile_decode.sh <tag> <bench args...>
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py "$@"
