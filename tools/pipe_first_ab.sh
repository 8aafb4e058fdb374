set -o pipefail
for r in 1 2 3; do
  for f in 131072 65536 32768; do
    HLC_PIPE_FIRST_CHUNK_VOTES=$f timeout -k 10 200 python tools/host_pipe.py --steps 10 --chunks 131072 --threads 4 --depths 3,4 > gpurun_out/pab_${f}_$r.txt 2>&1 || exit 1
    grep chunk_votes gpurun_out/pab_${f}_$r.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$r first=$f depth', d['depth'], round(d['votes_per_s']/1e6,2), 'M', d['outputs_equal_one_shot'])"
  done
done
