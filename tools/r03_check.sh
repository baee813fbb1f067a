#!/bin/bash
# round 3 GPU round trip: new tests, full suite, bench, k_map phase stamps, I-cache counters
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "200|python -u -m pytest tests/test_gpu_rccl.py tests/test_mr_workers.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1" \
  "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
  "150|python bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err" \
  "120|WCG_LIB=build/var/libwcg_stamps.so python bench.py --steps 3 --warmup 1 --no-verify --no-cpu-baseline --no-end-to-end > gpurun_out/stamps.json 2>gpurun_out/stamps.err" \
  "70|timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_map --output-format csv -d gpurun_out/icache -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-end-to-end > gpurun_out/icache.log 2>&1"
