# round 5: emit_asm storing a lane's tokens four at a time (16-byte stores; build/ab/lib_x4.so)
# against the in-tree 4-byte stores -- inflate A/B on B, D, E (output sha1 must match), then the
# Huffman phase probe at the X4 sources for the emit pass's share.
set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05m B 4000000 x4 || exit 1
timeout -k 10 600 bash tools/gpu_round.sh ab r05m D 25000 x4 || exit 2
timeout -k 10 600 bash tools/gpu_round.sh ab r05m E 4000000 x4 || exit 3
echo done
