#!/bin/bash
# One parametrised GPU-box runner (replaces the round-2 one-off gpu_*.sh wrappers).
#
#   tools/gpu_run.sh STEP [STEP ...]        (run through gpurun from the repo root)
#
# STEP forms (each runs under its own `timeout -k 10`, output under gpurun_out/; the first
# failing step ends the run with its exit code):
#   tests[=PATHS]            pytest -m gpu (default: the whole GPU suite)        -> pytest_gpu_<n>.log
#   smoke                    __graft_entry__.smoke()                             -> smoke.log
#   bench[=BENCH_ARGS]       python bench.py BENCH_ARGS                          -> bench_<n>.log
#   prof=TAG[=BENCH_ARGS]    rocprofv3 kernel trace of bench.py + prof_summary   -> prof_TAG/, prof_TAG.md
#   py=SCRIPT[=ARGS]         python SCRIPT ARGS (tools, microbenchmarks)         -> py_<n>.log
# Example:  gpurun -- 'bash tools/gpu_run.sh tests smoke bench prof=final="--steps 13 --warmup 3"'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
n=0
for step in "$@"; do
  n=$((n + 1))
  # never overwrite an earlier invocation's logs in the same call (A/B runs chain invocations)
  while compgen -G "gpurun_out/*_$n.log" > /dev/null; do n=$((n + 1)); done
  kind=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  case "$kind" in
    tests)
      # tests=PATHS runs those files / node ids instead of the whole GPU suite
      timeout -k 10 1000 python -u -m pytest ${arg:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu_$n.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench)
      timeout -k 10 600 python bench.py $arg > gpurun_out/bench_$n.log 2>&1 ;;
    prof)
      tag=${arg%%=*}
      bargs=""
      [[ "$arg" == *=* ]] && bargs=${arg#*=}
      (cd /tmp && export TMPDIR=/tmp) && export TMPDIR=/tmp && \
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run \
        -- python3 bench.py $bargs > gpurun_out/prof_${tag}_bench.log 2>&1 && \
      python tools/prof_summary.py "$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -n 1)" \
        --layers 80 --md gpurun_out/prof_$tag.md > /dev/null ;;
    py)
      script=${arg%%=*}
      pargs=""
      [[ "$arg" == *=* ]] && pargs=${arg#*=}
      timeout -k 10 900 python -u $script $pargs > gpurun_out/py_$n.log 2>&1 ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  echo "[$rc] $step"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
