# round 5, late: check-bam -s and full-check over configs[2]'s 100.9 GiB file at the final kernel
# sources (streamed through HBM, sbh_check_stream).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 540 python3 -u tools/allpos_configC.py --file-gib 100 > gpurun_out/r05zv_allpos100.log 2>&1 || exit 1
timeout -k 10 560 python3 -u tools/allpos_configC.py --file-gib 100 --full > gpurun_out/r05zv_allpos100_full.log 2>&1 || exit 2
echo done
