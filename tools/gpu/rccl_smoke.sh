# 1-rank RCCL smoke (tools/rccl_smoke.py) through the same launcher as tests/test_gpu_rccl.py
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -c "
import os, sys
sys.path.insert(0, '.')
from spark_druid_olap_amd.utils.launch import spawn_ranks
env = dict(os.environ, MASTER_ADDR='127.0.0.1')
env.pop('SDO_GLOO_GPU', None)
sys.exit(spawn_ranks(1, [sys.executable, 'tools/rccl_smoke.py', '--out', 'gpurun_out/r6/rccl_smoke.json', '--sf', '${SF:-1}'], env=env))
" > gpurun_out/r6/rccl_smoke.log 2>&1
