#!/bin/bash
# Round-3 (through gpurun, from the repo root): tools/gpu_batch_r03v.sh then tools/gpu_batch_r03w.sh
# (cache-policy A/B of the frame assembly and of the unmask + UTF-8 kernel) in one call.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_batch_r03v.sh || exit 1
bash tools/gpu_batch_r03w.sh || exit 1
echo all done
