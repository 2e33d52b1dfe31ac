set -u
cd $GRAFT_REPO_ROOT
for b in 65536 65600 65472 66048; do
  timeout -k 10 120 python bench.py --precision f32_split --no-cpu-baseline --steps 10 --batch $b > gpurun_out/bb_$b.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/bb_$b.json').read().strip().splitlines()[-1]); print('B=$b', round(d['roofline']['kernel_ms'], 3), 'ms', round(d['value']/1e6, 2), 'M/s')"
done
timeout -k 10 120 python bench.py --no-cpu-baseline --no-split --steps 10 --batch 65600 > gpurun_out/bb_f32.json 2>/dev/null && python -c "import json; d=json.loads(open('gpurun_out/bb_f32.json').read().strip().splitlines()[-1]); print('f32 B=65600', round(d['roofline']['kernel_ms'], 3), 'ms', round(d['value']/1e6, 2), 'M/s')"
