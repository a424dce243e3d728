# round 5, late: k_huff's pass 1 stores its tokens (provisional slots in the upper half of the block's
# token region) and the emit pass copies the chains the repair rounds kept (SBH_HUFF_PROV) -- the
# inflate/check GPU tests first, the rest of the suite, then the inflate A/B against lib_pv0 (decode
# in the emit pass, as before) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_gpu_parity.py \
  > gpurun_out/r05zj_pytest_parity.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zj_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zj B 4000000 pv0 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zj D 25000 pv0 || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zj E 4000000 pv0 || exit 5
echo done
