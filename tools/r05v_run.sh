# round 5: re-measure pipelined batches of the bench step (k_huff / k_lz / k_eager on three
# streams) at the current kernels: one batch (default) vs 2 / 3 / 6 batches, ABAB.
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --no-full --no-e2e --steps 20 --warmup 3"
for r in 1 2; do
  for nb in 0 22924 15283 7642; do
    if [ $nb = 0 ]; then
      timeout -k 10 300 $B > gpurun_out/r05v_pipe1_$r.json 2>/dev/null || exit 1
    else
      SBH_PIPE_MIN_BLOCKS=$nb timeout -k 10 300 $B > gpurun_out/r05v_pipe${nb}_$r.json 2>/dev/null || exit 2
    fi
  done
done
echo done
