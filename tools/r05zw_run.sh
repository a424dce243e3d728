# round 5, late: literal-pair table entries and two-byte literal tokens (SBH_HUFF_PAIRS: one decode
# step and one token for two literal codes that fit the 10-bit window together) -- inflate tests,
# the GPU suite, the inflate A/B against lib_np0 (single literals) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_inflate_distance_gpu.py \
  tests/test_gpu_parity.py > gpurun_out/r05zw_pytest_inflate.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zw_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zw B 4000000 np0 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zw D 25000 np0 || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zw E 4000000 np0 || exit 5
echo done
