#!/bin/bash
# GPU suite + smoke + C2 bench (full line, CPU legs) + C2/C4 kernel traces + PMC passes (C2: k_map,
# k_agg; C4 1 GiB: its aggregation, sort and long-key kernels; the last pass of each is the MFMA
# counters)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
  "120|python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1" \
  "300|python bench.py > gpurun_out/bench_full.json 2>gpurun_out/bench_full.err" \
  "150|python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/bench_c4.json 2>gpurun_out/bench_c4.err" \
  "120|tools/prof_trace.sh gpurun_out/trace_c2 > gpurun_out/trace_c2.log 2>&1" \
  "150|tools/prof_trace.sh gpurun_out/trace_c4 --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/trace_c4.log 2>&1" \
  "300|tools/prof_pmc.sh gpurun_out/pmc_c2 'k_map|k_agg' > gpurun_out/pmc_c2.log 2>&1" \
  "500|tools/prof_pmc.sh gpurun_out/pmc_c4 'k_agg|k_rp|k_ss_|k_long_hash|k_long_agg|k_map|k_compact' --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/pmc_c4.log 2>&1"
