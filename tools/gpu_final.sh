#!/bin/bash
# Round-end measurements at HEAD (outputs tagged $2 under gpurun_out/), in parts that each fit one
# gpurun call:  tools/gpu_final.sh A|B TAG
#   A: pytest -m gpu, smoke(), the default bench line (CPU legs, end to end), its kernel trace,
#      C4 1 GiB bench line + kernel trace
#   B: C3 16 GiB on one GPU, the N = 2 self-launched bench through gloo, PMC passes (C2 k_map
#      traffic -> traffic file, C4 kernels), ingest probe
# (C4 at 64 GiB: tools/c4_full.py, a call of its own)
export TMPDIR=/tmp
P=$1; T=${2:-final}
C4="--workload c4_utf8_zipf_64gib --bytes 1073741824"
if [ "$P" == "A" ]; then
tools/gpu_steps.sh \
 "600|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1" \
 "120|python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$T.log 2>&1" \
 "400|python bench.py > gpurun_out/bench_full_$T.json 2> gpurun_out/bench_full_$T.err" \
 "300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c2_$T -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/trace_c2_$T.json" \
 "300|python bench.py $C4 --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > gpurun_out/c4_$T.json 2> gpurun_out/c4_$T.err" \
 "300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_c4_$T -o run -- python3 bench.py $C4 --steps 5 --warmup 2 --no-cpu-baseline --no-verify --no-end-to-end > gpurun_out/trace_c4_$T.json"
elif [ "$P" == "B" ]; then
tools/gpu_steps.sh \
 "400|python bench.py --workload c3_ascii_zipf_16gib --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > gpurun_out/c3_$T.json 2> gpurun_out/c3_$T.err" \
 "600|python bench.py --gpus 2 --dist-backend gloo --bytes 4294967296 --no-cpu-baseline --no-end-to-end > gpurun_out/n2_gloo_$T.json 2> gpurun_out/n2_gloo_$T.err" \
 "400|tools/prof_pmc.sh gpurun_out/pmc_c2_$T 'k_map|k_agg' > gpurun_out/pmc_c2_$T.log 2>&1" \
 "400|tools/prof_pmc.sh gpurun_out/pmc_c4_$T 'k_map|k_agg|k_rp|k_long|k_ss|k_fmt|k_tie' $C4 > gpurun_out/pmc_c4_$T.log 2>&1" \
 "200|python3 tools/ingest_probe.py > gpurun_out/ingest_$T.log 2>&1" \
 "200|rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/ingest_trace_$T -o run -- python3 tools/ingest_probe.py > gpurun_out/ingest_trace_$T.log 2>&1"
fi
