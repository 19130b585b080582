export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline 0 > gpurun_out/ab_bench1.json 2>/dev/null || exit 1
timeout -k 10 300 python -u -c "import sys; sys.path.insert(0,'tools'); import bench_configs as b; from hakai import mesh; b.run('C3', mesh.config_c3(v_end=5e5), 400, 200)" > gpurun_out/ab_cfg.json 2>/dev/null || exit 2
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline 0 > gpurun_out/ab_bench2.json 2>/dev/null || exit 3
python -c "
import json
for f in ['ab_bench1','ab_cfg','ab_bench2']:
    d=json.loads(open('gpurun_out/'+f+'.json').read().strip().splitlines()[-1])
    print(f, d.get('ms_per_step'), d.get('kernel_ms_per_step') or d['config'].get('kernel_ms_per_step'), d.get('roofline',{}).get('avg_launch_ms'))
"
