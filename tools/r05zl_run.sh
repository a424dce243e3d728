# round 5, late: provisional tokens with the lanes' 16-byte groups interleaved (a wave's stores of
# one group index contiguous) -- parity tests, then the inflate A/B against lib_pv0 on B, D, E, and
# the Huffman phase probe (lib_hp) on B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_gpu_parity.py \
  > gpurun_out/r05zl_pytest_parity.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zl B 4000000 pv0 || exit 3
AB_ROUNDS=1 timeout -k 10 600 bash tools/gpu_round.sh ab r05zlp B 4000000 hp || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zl D 25000 pv0 || exit 5
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zl E 4000000 pv0 || exit 6
echo done
