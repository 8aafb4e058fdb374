#!/bin/bash
# Round-6 measurement call: the driver's bench command (compact line + side file), the committed rocprof
# profile of it (tools/profile.sh r06), far-node staging A/B with placement facts (tools/numa_ab.py), and the
# N > 1 code path rehearsed on one GPU (gloo dry run with two ranks; RCCL at one rank).
set -o pipefail
mkdir -p gpurun_out/r06
export HLC_BENCH_DETAIL=$PWD/gpurun_out/r06/bench_detail.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06/bench.json 2> gpurun_out/r06/bench.err || { tail gpurun_out/r06/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06/bench.json
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06/n2_detail.json HLC_BENCH_BACKEND=gloo HLC_BENCH_SAME_GPU=1 timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py \
  --gpus 2 --steps 3 --warmup 1 --proposals 20000 > gpurun_out/r06/n2_gloo.json 2> gpurun_out/r06/n2_gloo.err || { tail gpurun_out/r06/n2_gloo.err; exit 1; }
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06/rccl1_detail.json HLC_BENCH_DIST=1 timeout -k 10 300 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py \
  --gpus 1 --config 4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06/rccl1.json 2> gpurun_out/r06/rccl1.err || { tail gpurun_out/r06/rccl1.err; exit 1; }
timeout -k 10 400 python -u tools/numa_ab.py --steps 10 --rounds 3 > gpurun_out/r06/numa_ab2.txt 2> gpurun_out/r06/numa_ab2.err || { tail gpurun_out/r06/numa_ab2.err; exit 1; }
bash tools/profile.sh r06 > gpurun_out/r06/profile.log 2>&1 || { tail -30 gpurun_out/r06/profile.log; exit 1; }
echo measure-done
