# round 5, final: PMC counters at the sources with literal pairs and carried k_lz chunks, then the
# GPU round (suite, bench B with its kernel summary, D, E) and the two-rank rehearsal on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 bash tools/gpu_round.sh pmc r05zz || exit 1
timeout -k 10 1000 bash tools/gpu_round.sh round r05zz || exit 2
timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-full --no-e2e \
  > gpurun_out/r05zz_bench_2rank_selflaunch_1gpu.json 2> gpurun_out/r05zz_bench_2rank.err || exit 3
echo done
