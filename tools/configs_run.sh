#!/bin/bash
# BASELINE configs 2 and 4 on one MI355X (bench.py lines into gpurun_out/cfg/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cfg
timeout -k 10 200 python bench.py --batch 10000 --no-cpu-baseline > gpurun_out/cfg/cfg2_b10k.json 2> gpurun_out/cfg/cfg2.err || exit 1
timeout -k 10 400 python bench.py --variant v6 --m 512 --n 2048 --layers 40 --batch 65536 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/cfg4.json 2> gpurun_out/cfg/cfg4.err || exit 1
