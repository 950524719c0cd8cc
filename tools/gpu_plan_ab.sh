# In-situ decode GEMM plan A/B: the whole 70B decode step with one projection's plan forced
# (BFLY_GEMM_PLAN), 1 GPU (BENCH_ARGS: extra bench.py arguments, e.g. another --model). Each line of gpurun_out/plan_ab.log: variant, ms/step, tok/s.
# Variants: lines "name N,K,Mbucket:kind,mt,nt,wk,bm,bn,sk" of the file given as $1
# ("name -" = the tuned table), default the round-2 first list below.
cd $GRAFT_REPO_ROOT
run() {
  name=$1; shift
  timeout -k 10 300 env "$@" python bench.py --steps 24 --warmup 3 $BENCH_ARGS < /dev/null > gpurun_out/plan_ab_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/plan_ab_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null)" >> gpurun_out/plan_ab.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
: > gpurun_out/plan_ab.log
if [ -n "$1" ]; then
  while read -r name plan; do
    [ -z "$name" ] && continue
    case "$name" in \#*) continue;; esac
    if [ "$plan" = "-" ]; then run "$name" BFLY_X=0; else run "$name" BFLY_GEMM_PLAN="$plan"; fi
  done < "$1"
  exit 0
fi
run base BFLY_X=0
run gu_dec256 BFLY_GEMM_PLAN="57344,8192,64:3,4,8,4,64,256,1"
run gu_dec224 BFLY_GEMM_PLAN="57344,8192,64:3,4,4,4,64,224,1"
run qkv_dec160 BFLY_GEMM_PLAN="10240,8192,64:3,5,8,4,64,160,4"
run o_dec128 BFLY_GEMM_PLAN="8192,8192,64:3,6,8,4,64,128,4"
run base2 BFLY_X=0
