export TMPDIR=/tmp
A='--workload c4_utf8_zipf_64gib --bytes 1073741824 --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end'
tools/gpu_steps.sh \
 "600|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_v6.log 2>&1" \
 "300|python bench.py $A > gpurun_out/c4_v6.json 2> gpurun_out/c4_v6.err" \
 "300|python bench.py --no-cpu-baseline --no-end-to-end > gpurun_out/c2_v6.json 2> gpurun_out/c2_v6.err" \
 "300|tools/prof_libs.sh gpurun_out/prof_v6 mit-6.824-2015_amd/wcg/libwcg.so" \
 "300|WCG_LONG_FORK=0 tools/prof_libs.sh gpurun_out/prof_v6s mit-6.824-2015_amd/wcg/libwcg.so" \
 "120|WCG_DEBUG=1 python3 bench.py --workload c4_utf8_zipf_64gib --bytes 1073741824 --steps 1 --warmup 1 --no-cpu-baseline --no-end-to-end --no-verify > gpurun_out/dbg_v6.json 2> gpurun_out/dbg_v6.err"
