# round 5: k_huff_big (40 KiB stage for blocks past k_huff's 24 KiB) -- the GPU suite, then the
# inflate A/B against the same library without it (lib_nobig.so) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zc_pytest_gpu.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zc B 4000000 nobig || exit 2
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zc D 25000 nobig || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zc E 4000000 nobig || exit 4
echo done
