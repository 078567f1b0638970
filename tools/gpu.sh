#!/bin/bash
# Build locally (abort on failure), then run a command on the GPU box.
set -e
cd /root/repo
python -m trigenicinteractionpredictor_amd.build > /tmp/build.log 2>&1 || { grep -E "error" -A3 /tmp/build.log | head -20; exit 1; }
timeout 2400 /usr/local/graft/bin/gpurun --timeout ${GPU_TIMEOUT:-1200} -- "$@" 2>&1 | tail -3
