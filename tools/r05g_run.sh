# round 5: the 16-bit code format between k_huff and k_lz -- the full GPU suite, inflate A/B
# against the round-4 token format (build/ab/lib_tok32.so), then the counter passes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05g_pytest_gpu.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05g B 4000000 tok32 || exit 2
timeout -k 10 600 bash tools/gpu_round.sh ab r05g D 25000 tok32 || exit 3
timeout -k 10 600 bash tools/gpu_round.sh ab r05g E 4000000 tok32 || exit 4
timeout -k 10 900 bash tools/gpu_round.sh pmc r05g --no-cpu-baseline --no-e2e --no-full --steps 2 --warmup 1 || exit 5
echo done
