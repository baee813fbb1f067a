#!/bin/bash
# round 3 GPU round trip: new tests, full suite, bench, k_map variants (build/var, WCG_LIB)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "200|python -u -m pytest tests/test_gpu_rccl.py tests/test_mr_workers.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1" \
  "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
  "150|python bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err" \
  "400|tools/variants.sh gpurun_out/var $VARIANTS > gpurun_out/variants.log 2>&1"
