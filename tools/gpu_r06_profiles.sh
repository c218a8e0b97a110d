#!/bin/bash
# r06 end-of-round evidence on the final build: the headline Gram's stats + PMC passes (r06_gram_pmc.json,
# read by bench.py for roofline.traffic), then rocprofv3 --stats of the C3 / C2 / C5 / C5-GGN lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_gram_pmc.sh r06 || exit 1
tools/gpu_stats.sh gpurun_out/r06/stats || exit 1
