# One GPU call made of several tools/gpu_round.sh steps, chained: the first failing step ends the
# call (each step keeps gpu_round.sh's own time limits).  Replaces the per-call tools/r05*_run.sh.
#   bash tools/gpu_seq.sh "tests r06a tests/test_threads_gpu.py" "bench r06a --facade-only --steps 5"
set -o pipefail
for step in "$@"; do
  echo "== $step"
  # shellcheck disable=SC2086
  bash tools/gpu_round.sh $step || { echo "step failed: $step"; exit 1; }
done
echo "all steps ok"
