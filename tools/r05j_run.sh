# round 5: the linear block chain (index without pointer-jumping rounds) and the host's O(log n)
# block-table handling -- the new chain tests first, the full GPU suite, the bench line and a
# step trace; then A/B probes: two-wave k_huff_tail (t128), k_full without its histogram /
# name-and-CIGAR tests / chain walks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu --timeout 120 --timeout-method thread -x -v tests/test_index_chain_gpu.py \
  > gpurun_out/r05j_pytest_chain.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests \
  > gpurun_out/r05j_pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/r05j_bench.json 2> gpurun_out/r05j_bench.err || exit 3
timeout -k 10 400 bash tools/gpu_round.sh trace r05j || exit 4
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05j B 4000000 t128 || exit 5
timeout -k 10 900 bash tools/gpu_round.sh fullab r05j 4000000 fnh ffo fnc || exit 6
echo done
