#!/bin/bash
# One parameterized script for GPU-box work (replaces the per-session gpu_r*.sh lease scripts).
#
#   tools/gpu.sh STEP [STEP ...]        e.g.  gpurun -- 'bash tools/gpu.sh smoke tests bench'
#
# Steps (each runs under its own time limit; the first failing step ends the call -- no retries):
#   smoke              __graft_entry__.smoke()
#   tests              pytest -m gpu (per-test thread timeout names a hung test)
#   test:PATH          one GPU test file / node id
#   bench              bench.py (SF, STEPS, WARMUP, MODEL env; extra args in BENCH_ARGS)
#   rocprof            kernel trace + stats of the bench's timed steps -> gpurun_out/prof/summary.txt
#   conc               tools/concurrency_bench.py (WORKLOAD fixed|varied|jmx, COALESCE, QPS, DUR, CLIENTS)
#   probe              tools/sql_probe.py (PROBE_ARGS)
#   pmc                PMC counter passes over tools/kbench_one.py (Q, SF); one pass per counter group
#   py:SCRIPT          python SCRIPT $PY_ARGS (a tool under tools/)
#   pyprof:SCRIPT      the same under rocprofv3 --kernel-trace --stats -> gpurun_out/pyprof_<name>/summary.txt
#                      (PYPROF_ARGS: extra tools/rocpd_summary.py options, e.g. --tail-ms 40 --timeline-ms 20)
#
# Outputs land in gpurun_out/<step>.* ; the tail of each is echoed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1

SF=${SF:-100}
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
MODEL=${MODEL:-tpch}

fail() { echo "[gpu.sh] step $1 failed (exit $2)"; tail -40 "$3"; exit 1; }

for step in "$@"; do
  case "$step" in
    smoke)
      timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || fail smoke $? gpurun_out/smoke.log
      tail -1 gpurun_out/smoke.log | cut -c1-200 ;;
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 || fail tests $? gpurun_out/pytest_gpu.log
      tail -2 gpurun_out/pytest_gpu.log ;;
    test:*)
      t="${step#test:}"
      timeout -k 10 600 python -u -m pytest "$t" -m gpu -x -v --timeout 150 --timeout-method thread \
        > gpurun_out/pytest_one.log 2>&1 || fail "$step" $? gpurun_out/pytest_one.log
      tail -2 gpurun_out/pytest_one.log ;;
    bench)
      tag=${TAG:-$MODEL}
      timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --model "$MODEL" --sf "$SF" --steps "$STEPS" --warmup "$WARMUP" \
        ${BENCH_ARGS:-} > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || fail bench $? gpurun_out/bench_$tag.err
      cut -c1-1500 gpurun_out/bench_$tag.json ;;
    rocprof)
      rm -rf gpurun_out/prof
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats \
        -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --model "$MODEL" --sf "$SF" --steps ${PSTEPS:-10} \
        --warmup 3 ${BENCH_ARGS:-} > "$R/gpurun_out/prof.log" 2>&1) || fail rocprof $? gpurun_out/prof.log
      DB=$(find gpurun_out/prof -name "*.db" | head -1)
      if [ -n "$DB" ]; then
        python tools/rocpd_summary.py "$DB" --tail-ms ${TAIL:-100} --top 40 --timeline-ms ${TL:-12} > gpurun_out/prof/summary.txt
      else
        python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof/summary.txt
      fi
      find gpurun_out/prof -name "*.db" -delete  # (summaries only: gpurun returns at most 64 MiB)
      head -50 gpurun_out/prof/summary.txt ;;
    conc)
      tag=${TAG:-${WORKLOAD:-fixed}}
      timeout -k 10 ${CONC_TIMEOUT:-300} python tools/concurrency_bench.py --sf "$SF" --clients ${CLIENTS:-64} \
        --procs ${PROCS:-16} --qps ${QPS:-0} --duration ${DUR:-20} --workload ${WORKLOAD:-fixed} \
        --coalesce ${COALESCE:-off} ${CONC_ARGS:-} > gpurun_out/conc_$tag.json 2> gpurun_out/conc_$tag.log \
        || fail conc $? gpurun_out/conc_$tag.log
      cut -c1-1200 gpurun_out/conc_$tag.json ;;
    probe)
      timeout -k 10 400 python tools/sql_probe.py ${PROBE_ARGS:-} > gpurun_out/probe.txt 2>&1 || fail probe $? gpurun_out/probe.txt
      grep -v "^$" gpurun_out/probe.txt | tail -${PROBE_TAIL:-40} ;;
    pmc)
      i=0
      for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" \
                 "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "FETCH_SIZE"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --output-format csv \
          -d "$R/gpurun_out/pmc$i" -o p -- python3 "$R/tools/kbench_one.py" --sf ${PSF:-$SF} --query "${Q:-TPCH Q1}" \
          --iters 3 > "$R/gpurun_out/pmc$i.log" 2>&1) || fail pmc $? gpurun_out/pmc$i.log
      done
      python tools/pmc_summary.py gpurun_out "${PMC_FILT:-sdo_}" "pmc[0-9]*" > gpurun_out/pmc_summary.txt 2>&1 || true
      rm -rf gpurun_out/pmc[0-9]*  # (the per-pass CSVs exceed what gpurun copies back; the summary stays)
      tail -40 gpurun_out/pmc_summary.txt ;;
    py:*)
      s="${step#py:}"
      b=$(basename "$s" .py)
      timeout -k 10 ${PY_TIMEOUT:-400} python "$s" ${PY_ARGS:-} > gpurun_out/py_$b.txt 2>&1 || fail "$step" $? gpurun_out/py_$b.txt
      grep -v "^$" gpurun_out/py_$b.txt | tail -${PY_TAIL:-40} ;;
    pyprof:*)
      s="${step#pyprof:}"
      b=$(basename "$s" .py)
      rm -rf gpurun_out/pyprof_$b
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${PY_TIMEOUT:-400} rocprofv3 --kernel-trace --stats \
        -d "$R/gpurun_out/pyprof_$b" -o run -- python3 "$R/$s" ${PY_ARGS:-} > "$R/gpurun_out/pyprof_$b.log" 2>&1) \
        || fail "$step" $? gpurun_out/pyprof_$b.log
      DB=$(find gpurun_out/pyprof_$b -name "*.db" | head -1)
      if [ -n "$DB" ]; then
        python tools/rocpd_summary.py "$DB" --top 30 ${PYPROF_ARGS:-} > gpurun_out/pyprof_$b/summary.txt
      else
        python tools/prof_summary.py gpurun_out/pyprof_$b > gpurun_out/pyprof_$b/summary.txt
      fi
      find gpurun_out/pyprof_$b -name "*.db" -delete
      head -40 gpurun_out/pyprof_$b/summary.txt ;;
    *)
      echo "[gpu.sh] unknown step $step"; exit 2 ;;
  esac
done
