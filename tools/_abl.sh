set -o pipefail
export TMPDIR=/tmp
ABL="0 3 4 6 8 9" bash tools/ablate.sh > gpurun_out/abl.log 2>&1; cat gpurun_out/abl.log
