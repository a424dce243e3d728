# round 5, late: the too-far-back distance test moved from the emit pass (6 instructions per code)
# to k_lz (once per match token; SBH_EMIT_NOCHK) -- the new distance tests, the whole GPU suite,
# then the inflate A/B against lib_chk (the test in the emit pass, as before) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -v tests/test_inflate_distance_gpu.py \
  > gpurun_out/r05zn_pytest_distance.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zn_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zn B 4000000 chk || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zn D 25000 chk || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zn E 4000000 chk || exit 5
echo done
