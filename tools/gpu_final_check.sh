# Round-end style check: full GPU test suite, smoke, 1-GPU bench, and a decode kernel trace.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
step timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
step timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
step timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 bench.py --steps 13 --warmup 3 > gpurun_out/prof_final_bench.log 2>&1
