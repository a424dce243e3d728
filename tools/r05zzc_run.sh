# round 5, final: k_lz's pointer pass at 6848 bytes (the most three workgroups per CU allow) and at
# 6400, against the in-tree 6656, now that chunks end at their pass cut -- inflate A/B on B, D, E.
set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05zzc B 4000000 cap68 cap64 || exit 1
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zzc D 25000 cap68 cap64 || exit 2
AB_ROUNDS=2 timeout -k 10 600 bash tools/gpu_round.sh ab r05zzc E 4000000 cap68 cap64 || exit 3
echo done
