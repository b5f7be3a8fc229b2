#!/bin/bash
# GPU box: SSB and headline A/B on the time-key LUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for L in 1 0; do
SDO_TIME_LUT=$L timeout -k 10 170 python bench.py --model ssb --steps 5 --warmup 2 --verbose > gpurun_out/ssb_lut$L.json 2> gpurun_out/ssb_lut$L.err || { tail -30 gpurun_out/ssb_lut$L.err; exit 1; }
echo "lut=$L ssb $(cut -c50-90 gpurun_out/ssb_lut$L.json)"
SDO_TIME_LUT=$L timeout -k 10 170 python bench.py --steps 10 --warmup 3 --verbose > gpurun_out/h_lut$L.json 2> gpurun_out/h_lut$L.err || { tail -30 gpurun_out/h_lut$L.err; exit 1; }
echo "lut=$L headline $(cut -c50-100 gpurun_out/h_lut$L.json)"
done
