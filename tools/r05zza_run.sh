# round 5, final: fill_ptables joins literal pairs from the single entries in LDS (SBH_PAIRS_LDS)
# instead of a second canonical lookup per entry -- inflate tests, the GPU suite, the inflate A/B
# against lib_pl0 (the second lookup) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_inflate_distance_gpu.py \
  tests/test_gpu_parity.py > gpurun_out/r05zza_pytest_inflate.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zza_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zza B 4000000 pl0 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zza D 25000 pl0 || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zza E 4000000 pl0 || exit 5
echo done
