# round 5, final: bench lines B, D, E with the counter summary of these sources committed
# (traffic_matches_kernels) -- the same sources as r05zz's round.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r05zzb_bench.json 2> gpurun_out/r05zzb_bench.err || exit 1
timeout -k 10 300 python -u bench.py --config D --no-cpu-baseline --no-full --no-e2e > gpurun_out/r05zzb_benchD.json \
  2> gpurun_out/r05zzb_benchD.err || exit 2
timeout -k 10 300 python -u bench.py --config E --no-cpu-baseline --no-full --no-e2e > gpurun_out/r05zzb_benchE.json \
  2> gpurun_out/r05zzb_benchE.err || exit 3
echo done
