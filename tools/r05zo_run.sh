# round 5, late: the decode loops address the tables from vt (tables at LDS address 0:
# SBH_HUFF_TAB0) and the emit pass drops its token / byte counters (they fed only the distance
# test, now k_lz's) -- inflate tests, the whole GPU suite, the inflate A/B against lib_tb0 (the
# previous commit's loops) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_inflate_distance_gpu.py \
  tests/test_gpu_parity.py > gpurun_out/r05zo_pytest_inflate.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zo_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zo B 4000000 tb0 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zo D 25000 tb0 || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zo E 4000000 tb0 || exit 5
echo done
