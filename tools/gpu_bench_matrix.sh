# 1-GPU bench matrix (session 5): Mixtral 8x7B B=64, Llama-3-70B B=128 / B=16 / B=1, Llama-3-8B B=64.
cd $GRAFT_REPO_ROOT
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 32 --warmup 4 --out gpurun_out/m_mixtral_b64.json > gpurun_out/m_mixtral_b64.log 2>&1
step timeout -k 10 400 python bench.py --batch-per-gpu 128 --steps 32 --warmup 4 --out gpurun_out/m_70b_b128.json > gpurun_out/m_70b_b128.log 2>&1
step timeout -k 10 400 python bench.py --batch-per-gpu 16 --steps 32 --warmup 4 --out gpurun_out/m_70b_b16.json > gpurun_out/m_70b_b16.log 2>&1
step timeout -k 10 400 python bench.py --batch-per-gpu 1 --steps 32 --warmup 4 --out gpurun_out/m_70b_b1.json > gpurun_out/m_70b_b1.log 2>&1
step timeout -k 10 400 python bench.py --model llama3-8b --steps 64 --warmup 4 --out gpurun_out/m_8b_b64.json > gpurun_out/m_8b_b64.log 2>&1
