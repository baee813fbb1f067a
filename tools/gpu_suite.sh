#!/bin/bash
# GPU suite: tests, smoke, C2 bench, C4 1 GiB bench, C4 kernel trace (outputs tagged $1).
# Each step under its own limit; stops at the first fault/timeout.
export TMPDIR=/tmp
TAG=${1:-v1}
tools/gpu_steps.sh \
 "600|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1" \
 "120|python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1" \
 "300|python bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/c2_$TAG.json 2> gpurun_out/c2_$TAG.err" \
 "300|python bench.py --workload c4_utf8_zipf_64gib --bytes 1073741824 --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err" \
 "300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4trace_$TAG -o run -- python3 bench.py --workload c4_utf8_zipf_64gib --bytes 1073741824 --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-end-to-end"
