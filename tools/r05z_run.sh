# round 5: the ring k_lz by default -- full GPU suite, bench B / D / E, then A/B of two tokens per
# thread (1024-token chunks, no VGPR spills at 80) against three.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05z_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r05z_bench.json 2> gpurun_out/r05z_bench.err || exit 2
timeout -k 10 300 python -u bench.py --config D --no-cpu-baseline --no-full --no-e2e > gpurun_out/r05z_benchD.json 2>/dev/null || exit 3
timeout -k 10 300 python -u bench.py --config E --no-cpu-baseline --no-full --no-e2e > gpurun_out/r05z_benchE.json 2>/dev/null || exit 4
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05z B 4000000 tpt2 || exit 5
timeout -k 10 600 bash tools/gpu_round.sh ab r05z D 25000 tpt2 || exit 6
timeout -k 10 600 bash tools/gpu_round.sh ab r05z E 4000000 tpt2 || exit 7
echo done
