# Bench A/B of the in-tree library against spark-bam_amd/build/ab/lib_$2.so (ABAB), config-B line
# without the side measurements.  usage: bash tools/lib_ab.sh TAG VARIANT [bench args...]
set -o pipefail
T=$1; V=$2; shift 2
B="python -u bench.py --no-cpu-baseline --no-full --no-e2e --steps 10 $*"
for r in 1 2; do
  SBH_LIB_PATH=spark-bam_amd/build/ab/lib_$V.so timeout -k 10 300 $B > gpurun_out/${T}_libab_${V}_$r.json 2>/dev/null || exit 3
  timeout -k 10 300 $B > gpurun_out/${T}_libab_intree_$r.json 2>/dev/null || exit 4
done
