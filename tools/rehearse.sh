#!/bin/bash
# Multi-rank bench.py rehearsals on ONE GPU: N ranks share cuda:0 over gloo (RCCL refuses two
# ranks on one device), small models, every layout the 8-GPU driver run can pick. Exercises the
# preflight, the partitioner, the program-driven stage execution (sync and async pipeline),
# the IPC all-reduce and the IPC EP exchange; each run under its own time limit, the first
# failure ends the script.
#   tools/rehearse.sh [MODEL:N:PLAN ...]   -> gpurun_out/rehearse_<model>_<plan>.log
# REHEARSE_ARGS replaces the default bench sizes (e.g. the real Llama-3-70B at its default batch:
#   REHEARSE_ARGS="--steps 8 --warmup 2 --prompt-len 256" tools/rehearse.sh llama3-70b:2:tp2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export BFLY_DIST_BACKEND=gloo
runs=("$@")
[ ${#runs[@]} -eq 0 ] && runs=(llama-small:8:auto llama-small:8:tp2xpp4 llama-small:4:pp4 llama-small:8:tp8
                                mixtral-tiny:4:ep4 mixtral-8x7b:8:ep8)
for r in "${runs[@]}"; do
  IFS=: read -r model n plan <<< "$r"
  log=gpurun_out/rehearse_${model}_${n}_${plan}.log
  timeout -k 10 420 python -m butterfly_amd launch -n "$n" -- python bench.py --gpus "$n" --model "$model" \
    --plan "$plan" ${REHEARSE_ARGS:---steps 8 --warmup 2 --batch-per-gpu 8 --prompt-len 64} --no-probe > "$log" 2>&1
  rc=$?
  grep -h '"metric"' "$log" | head -n 1 | cut -c1-220
  echo "[$rc] $model n=$n plan=$plan"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
