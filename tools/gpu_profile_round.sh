# Kernel trace of the 1-GPU Llama-3-70B bench (prefill + 13 decode steps): per-kernel stats.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2 -o run -- python3 bench.py --steps 13 --warmup 3 > gpurun_out/prof_r2_bench.log 2>&1
echo "[$?] profile"
