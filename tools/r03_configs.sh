#!/bin/bash
# Round-3 measurement set on one MI355X: BASELINE configs 2, 4, 5 bench lines, every variant at
# the headline shape, and rocprofv3 kernel stats of config 2 (B = 10,000)  -> gpurun_out/r03/
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/r03
timeout -k 10 200 python bench.py --batch 10000 --no-cpu-baseline > gpurun_out/r03/cfg2_b10k.json 2> gpurun_out/r03/cfg2.err || exit 1
timeout -k 10 400 python bench.py --variant v6 --m 512 --n 2048 --layers 40 --batch 65536 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03/cfg4.json 2> gpurun_out/r03/cfg4.err || exit 1
timeout -k 10 200 python bench.py --precision bf16 --m 1024 --n 4096 --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03/cfg5.json 2> gpurun_out/r03/cfg5.err || exit 1
timeout -k 10 400 python tools/bench_variants.py > gpurun_out/r03/variants.jsonl 2> gpurun_out/r03/variants.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03/cfg2prof -o run -- python3 $R/bench.py --batch 10000 --steps 10 --warmup 3 --no-split --no-cfg3 --no-cpu-baseline > $R/gpurun_out/r03/cfg2prof.log 2>&1 || exit 1
