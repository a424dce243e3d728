set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 bash tools/calib_counters.sh gpurun_out/r05e_calib > gpurun_out/r05e_calib.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 900 bash tools/gpu_round.sh ab r05e B 4000000 t768 || exit 2
timeout -k 10 600 bash tools/gpu_round.sh ab r05e D 25000 t768 || exit 3
timeout -k 10 600 python3 -u tools/allpos_configC.py --file-gib 100 > gpurun_out/r05e_allpos100.log 2>&1 || exit 4
timeout -k 10 900 python3 -u tools/allpos_configC.py --file-gib 100 --full > gpurun_out/r05e_allpos100_full.log 2>&1 || exit 5
echo done
