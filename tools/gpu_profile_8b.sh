# Kernel trace of the 1-GPU Llama-3-8B bench (B=64, 1024-token prompts).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 bench.py --model llama3-8b --steps 32 --warmup 4 > gpurun_out/bench_8b.log 2>&1
echo "[$?] bench 8b"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_8b -o run -- python3 bench.py --model llama3-8b --steps 13 --warmup 3 > gpurun_out/prof_8b_bench.log 2>&1
echo "[$?] profile 8b"
