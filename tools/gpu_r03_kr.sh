#!/bin/bash
# round 3: k_map dword key reads (kr4) vs 8-byte pairs (kr0); GPU suite; C4 1 GiB; bench N=2
# through gloo on the one GPU (a rehearsal of the N>1 code path, 4 GiB of C3)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|tools/bench_libs.sh gpurun_out/kr --args '--steps 30 --warmup 15 --no-cpu-baseline --no-end-to-end' build/var/libwcg_kr4.so build/var/libwcg_kr0.so build/var/libwcg_kr4.so build/var/libwcg_kr0.so > gpurun_out/kr.txt 2>&1" \
 "400|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1" \
 "200|python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --workload c4_utf8_zipf_64gib --bytes 1073741824 > gpurun_out/c4.json 2> gpurun_out/c4.err" \
 "300|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 3 --bytes 4294967296 > gpurun_out/n2.json 2> gpurun_out/n2.err"
