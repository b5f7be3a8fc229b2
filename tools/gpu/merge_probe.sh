# one-rank forced-collective merge probe (tools/merge_probe.py) through the RCCL smoke's launcher
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
for Q in "TPCH Q3"; do
timeout -k 10 300 python -u -c "
import os, sys
sys.path.insert(0, '.')
from spark_druid_olap_amd.utils.launch import spawn_ranks
env = dict(os.environ, MASTER_ADDR='127.0.0.1')
env.pop('SDO_GLOO_GPU', None)
sys.exit(spawn_ranks(1, [sys.executable, 'tools/merge_probe.py', '--out', 'gpurun_out/r6/merge_probe.json', '--sf', '${SF:-1}', '--query', '$Q'], env=env))
" > gpurun_out/r6/merge_probe.log 2>&1 || exit $?
done
