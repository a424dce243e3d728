# A/B of the host wait mode (SBH_SCHED) on the config-B bench line, alternating (ABAB).
set -o pipefail
B="python -u bench.py --no-cpu-baseline --no-full --no-e2e --steps 10"
for r in 1 2; do
  timeout -k 10 300 $B > gpurun_out/${1}_sched_default_$r.json 2>/dev/null || exit 3
  SBH_SCHED=spin timeout -k 10 300 $B > gpurun_out/${1}_sched_spin_$r.json 2>/dev/null || exit 4
done
