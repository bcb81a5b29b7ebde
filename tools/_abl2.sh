set -o pipefail
export TMPDIR=/tmp
mkdir -p abl gpurun_out
cd fem-libraries_amd/csrc
for k in 0 6; do /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -DFA_ABL=$k -o ../../abl/libfemasm_abl$k.so femasm.hip & done; wait
cd ../..
for k in 0 6; do for m in 0 1 2 4; do
  FEMASM_GATHER_GRID_MULT=$m FEMASM_LIB=$PWD/abl/libfemasm_abl$k.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/x.json 2> gpurun_out/x.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/x.json'));print('abl $k mult $m', d['value'], d['roofline']['launch_ms'])"
done; done
