#!/bin/bash
# round 6 batch 20: cross-XCD stores into one 128-B line (tools/probe/line_share_probe.hip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/probe/line_share_probe 20 > gpurun_out/b20_share.txt 2>&1; rc=$?; cat gpurun_out/b20_share.txt; exit $rc
