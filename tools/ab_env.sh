#!/bin/bash
# A/B of one environment switch of the default build (GPU box): parity with the switch on, then
# alternating short benches.  Usage: tools/ab_env.sh VAR "valA" "valB"
set -o pipefail
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3
env $VAR=$A timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py -k "parity or config2 or golden or edge" -x -q -m gpu > gpurun_out/abenv_parity.log 2>&1 || { tail -30 gpurun_out/abenv_parity.log; exit 1; }
tail -1 gpurun_out/abenv_parity.log
for round in 1 2; do
  for v in "$A" "$B"; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config3 --no-wire --no-stream --no-e2e > gpurun_out/abenv_$v.json 2> gpurun_out/abenv_$v.err || { tail gpurun_out/abenv_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abenv_$v.json'));print('$round $VAR=$v', round(d['value']), 'votes/s rec_ms', round(d['roofline']['kernel_ms_avg'],3), 'step_ms', round(d['ms_per_step'],3))"
  done
done
