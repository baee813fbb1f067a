#!/bin/bash
# round 3: bench N=2 through gloo on the one GPU (4 GiB of C3: the N>1 code path with its stage
# timings), then C4 at full size (64 GiB, 8 calls of 8 GiB, verified exactly)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 3 --bytes 4294967296 > gpurun_out/n2.json 2> gpurun_out/n2.err" \
 "900|python -u tools/c4_full.py --jobs 2 --out gpurun_out/c4_full.json > gpurun_out/c4_full.log 2>&1"
