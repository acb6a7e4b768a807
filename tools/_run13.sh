set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lfq_proj.py tests/test_gpu_lfq_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t13.log 2>&1; rc=$?; tail -3 gpurun_out/t13.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/t13.log | head -30; exit $rc; }
for lib in "" "_ablate/c1/libdctae.so"; do
  DCTAE_LIBRARY=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stats --no-model > gpurun_out/b13.log 2>&1 || { tail -20 gpurun_out/b13.log; exit 1; }
  grep '^{' gpurun_out/b13.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); oc=d['other_configs']; lp=oc.get('lfq_projections',{})
print('[$lib]', d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, 'lfqp', lp.get('ms_per_step'), {k:v['total_ms'] for k,v in lp.get('kernels',{}).items()}, 'dec', (lp.get('decode') or {}).get('ms_per_step'), 'cfg2', oc.get('config2',{}).get('ms_per_step'), 'cfg4', oc.get('config4',{}).get('ms_per_step'))"
done
