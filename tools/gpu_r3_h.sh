#!/bin/bash
# Re-entry check of the round-3 build: whole GPU suite + smoke + default bench, then every config's bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/full_check.sh || exit $?
bash tools/gpu_r3_g.sh
