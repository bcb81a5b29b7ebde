#!/bin/bash
# gpu_d (tests + A/B benches) then gpu_e (phase clocks)
set -o pipefail
./tools/r4/gpu_d.sh && ./tools/r4/gpu_e.sh
