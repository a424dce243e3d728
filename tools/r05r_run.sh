# round 5: chain marking by peeling (and the tail's chain proof reused) -- the chain tests
# first, the full GPU suite, then bench lines E (whose false-positive bait takes the marking
# path) and B, and E's kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -v \
  tests/test_gpu_parity.py -k "chain" > gpurun_out/r05r_pytest_chain.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05r_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --config E --no-cpu-baseline --no-full --no-e2e > gpurun_out/r05r_benchE.json \
  2> gpurun_out/r05r_benchE.err || exit 3
timeout -k 10 300 python -u bench.py > gpurun_out/r05r_bench.json 2> gpurun_out/r05r_bench.err || exit 4
timeout -k 10 400 bash tools/gpu_round.sh prof r05rE --config E --steps 5 --warmup 2 --no-cpu-baseline --no-full --no-e2e || exit 5
echo done
