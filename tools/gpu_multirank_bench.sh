# The driver's N = 4 / 8 bench layouts (dp2xtp2, dp4xtp2) rehearsed with ranks sharing one GPU
# over gloo (RCCL refuses two ranks per device): llama-small, hipGraph decode, IPC all-reduce.
cd $GRAFT_REPO_ROOT
export BFLY_DIST_BACKEND=gloo
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python -m butterfly_amd launch -n 4 -- python bench.py --gpus 4 --model llama-small --plan dp2xtp2 --steps 8 --warmup 2 --batch-per-gpu 8 --prompt-len 64 > gpurun_out/mr_dp2xtp2.log 2>&1
step timeout -k 10 500 python -m butterfly_amd launch -n 8 -- python bench.py --gpus 8 --model llama-small --plan dp4xtp2 --steps 8 --warmup 2 --batch-per-gpu 8 --prompt-len 64 > gpurun_out/mr_dp4xtp2.log 2>&1
