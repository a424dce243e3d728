# round 5: k_lz's block image as a ring (32 KiB of history + one 6656-byte pass, flushed to U pass
# by pass): 3 workgroups per CU at 80 VGPRs (lib_ring.so) and the ring alone at 2 per CU
# (lib_ring5.so) against the in-tree 64 KiB image; output sha1 must match.
set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05y B 4000000 ring ring5 || exit 1
timeout -k 10 600 bash tools/gpu_round.sh ab r05y D 25000 ring ring5 || exit 2
timeout -k 10 600 bash tools/gpu_round.sh ab r05y E 4000000 ring ring5 || exit 3
echo done
