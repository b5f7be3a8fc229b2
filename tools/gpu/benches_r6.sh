# Round-6 measurements: the headline bench (SF100), the SF125 single-shard proxy of the 8-GPU
# config and SSB SF37.5, each on a fresh process.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench_headline.json 2> gpurun_out/r6/bench_headline.err &&
timeout -k 10 400 python bench.py --sf 125 --steps 20 --warmup 5 > gpurun_out/r6/bench_sf125.json 2> gpurun_out/r6/bench_sf125.err &&
timeout -k 10 400 python bench.py --model ssb --sf 37.5 --steps 10 --warmup 3 > gpurun_out/r6/bench_ssb375.json 2> gpurun_out/r6/bench_ssb375.err
