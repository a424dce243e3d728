# round 5, late: k_huff's prologue in one memory round trip (header record + stage loaded
# together), k_huff_tail's table entries / tail record / stage window in two, and k_lz's next
# chunk of tokens issued during the last pass's second half granule (SBH_LZ_PREFETCH=2) -- the
# GPU suite, then the inflate A/B against lib_l0 (both load changes off), lib_lt0 (tail change
# off) and lib_p2 (the k_lz prefetch) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zh_pytest_gpu.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zh B 4000000 l0 lt0 p2 || exit 2
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zh D 25000 l0 p2 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zh E 4000000 l0 p2 || exit 4
echo done
