# round 5: k_eager look-ahead 4096 (in-tree) vs 3072 / 2048 bytes (build/ab/lib_ela*.so): eager
# stage time and record counts on B, D, E.
set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05x B 4000000 ela3k ela2k || exit 1
timeout -k 10 600 bash tools/gpu_round.sh ab r05x D 25000 ela3k ela2k || exit 2
timeout -k 10 600 bash tools/gpu_round.sh ab r05x E 4000000 ela3k ela2k || exit 3
echo done
