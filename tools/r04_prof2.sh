#!/bin/bash
# Headline-only rocprofv3 passes (tools/profile.sh, 20 timed steps) -> gpurun_out/r04p/prof
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && STEPS=20 bash tools/profile.sh || exit 1
rm -rf gpurun_out/r04p && mkdir -p gpurun_out/r04p && cp -r gpurun_out/prof gpurun_out/r04p/prof
echo done
