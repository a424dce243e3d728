# round 5, late: k_lz chunks that end at their pass cut (the next chunk starts at the cut token:
# SBH_LZ_CARRY) with and without literal-pair tokens (SBH_HUFF_PAIRS) -- inflate tests and the GPU
# suite with both on, then the inflate A/B against lib_c0p1 (pairs, no carry), lib_c1p0 (carry,
# no pairs) and lib_c0p0 (neither: the committed kernels) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_inflate_distance_gpu.py \
  tests/test_gpu_parity.py > gpurun_out/r05zy_pytest_inflate.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zy_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 1000 bash tools/gpu_round.sh ab r05zy B 4000000 c0p1 c1p0 c0p0 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zy D 25000 c0p1 c1p0 c0p0 || exit 4
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zy E 4000000 c0p1 c1p0 c0p0 || exit 5
echo done
