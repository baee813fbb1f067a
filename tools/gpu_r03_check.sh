#!/bin/bash
# round 3: GPU suite, C2 + C4 bench lines and a C2 kernel trace at the working tree
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "150|python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err" \
 "200|python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err" \
 "150|tools/prof_trace.sh gpurun_out/trace_c2 > gpurun_out/trace_c2.log 2>&1" || exit $?
tools/gpu_steps.sh \
 "250|tools/bench_libs.sh gpurun_out/k1 build/var/libwcg_nospeck1.so build/var/libwcg_speck1.so build/var/libwcg_nospeck1.so build/var/libwcg_speck1.so > gpurun_out/speck1_c2.txt 2>&1" \
 "300|tools/bench_libs.sh gpurun_out/k1c4 --args '--steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824' build/var/libwcg_nospeck1.so build/var/libwcg_speck1.so > gpurun_out/speck1_c4.txt 2>&1"
