# round 5, late: emit_asm takes its token-start mask from the last code's length-code mask (one scalar op
# instead of a compare: SBH_EMIT_SA_SALU), and a two-token store queue (SBH_EMIT_X4=2) -- inflate tests,
# the GPU suite, the inflate A/B against lib_sa0 (the compare) and lib_x2 (8-byte stores) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -q tests/test_inflate_distance_gpu.py \
  tests/test_gpu_parity.py > gpurun_out/r05zt_pytest_inflate.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zt_pytest_gpu.log 2>&1 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zt B 4000000 sa0 x2 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zt D 25000 sa0 x2 || exit 4
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zt E 4000000 sa0 x2 || exit 5
echo done
