# round 5, late: the Huffman phase probe with the provisional-token emit (lib_hp) and without
# (lib_hp0), config B, 4 M records: where the provisional path's time goes.
set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=1 timeout -k 10 600 bash tools/gpu_round.sh ab r05zk B 4000000 hp hp0 || exit 1
echo done
