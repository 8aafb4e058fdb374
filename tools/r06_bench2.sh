set -o pipefail
mkdir -p gpurun_out/r06
for i in 1 2; do
HLC_BENCH_DETAIL=$PWD/gpurun_out/r06/bench_c${i}_detail.json timeout -k 10 300 python bench.py > gpurun_out/r06/bench_c$i.json 2> gpurun_out/r06/bench_c$i.err || { tail gpurun_out/r06/bench_c$i.err; exit 1; }
python tools/bench_summary.py gpurun_out/r06/bench_c$i.json
done
