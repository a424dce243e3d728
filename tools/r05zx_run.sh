# round 5, late: literal pairs with 448-thread k_lz workgroups (1344-token chunks, so that a chunk
# of two-byte literal tokens still fits one pointer pass) -- the inflate A/B of the in-tree library
# (pairs, 512 threads) against lib_np0 (no pairs), lib_p448 (pairs, 448) and lib_np448 (no pairs,
# 448) on B, D, E.
set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=2 timeout -k 10 1000 bash tools/gpu_round.sh ab r05zx B 4000000 np0 p448 np448 || exit 1
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zx D 25000 np0 p448 np448 || exit 2
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zx E 4000000 np0 p448 np448 || exit 3
echo done
