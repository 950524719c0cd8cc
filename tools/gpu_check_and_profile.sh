# Full GPU test suite, then a rocprofv3 kernel trace of the 1-GPU Llama-3-70B bench
# (decode window summarised by tools/prof_summary.py on the host).
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
step timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2c -o run -- python3 bench.py --steps 13 --warmup 3 > gpurun_out/prof_r2c_bench.log 2>&1
