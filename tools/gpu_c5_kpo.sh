cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in def k200 def k200; do
  if [ $v = k200 ]; then export SHP_SW_KPO=200; else unset SHP_SW_KPO; fi
  timeout -k 10 300 python3 -u bench.py --config 5 --no-cpu-baseline --latency-batches 0 --steps 5 --warmup 2 > gpurun_out/c5_$v.log 2>&1 || { tail -20 gpurun_out/c5_$v.log; exit 1; }
  grep '^{' gpurun_out/c5_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernel_ms_per_launch'); print('$v', round(d['ms_per_step'],3), round(d['value']/1e9,2), {a:round(b,3) for a,b in (k or {}).items()})"
done
