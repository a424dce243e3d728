# round 5, late: the decode loops read the stage dword after a lane's 64-bit window only when the
# lane moves into the next dword (SBH_HUFF_NXLAZY) -- the GPU suite, then the inflate A/B against
# lib_nx0 (a read every code, as before) and lib_wb1 (k_lz chase write-back only in rounds the
# lane goes on, SBH_LZ_WB_CONT) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05zi_pytest_gpu.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zi B 4000000 nx0 wb1 || exit 2
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zi D 25000 nx0 wb1 || exit 3
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zi E 4000000 nx0 wb1 || exit 4
echo done
