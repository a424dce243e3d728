# One GPU call: inflate A/B of the variants named on the command line (spark-bam_amd/build/ab/lib_<v>.so)
# usage: bash tools/gpu_ab.sh TAG RECORDS v1 v2 ...
set -o pipefail
T=$1; N=$2; shift 2
mkdir -p gpurun_out
L=""
for v in "$@"; do L="$L spark-bam_amd/build/ab/lib_$v.so"; done
timeout -k 10 400 python -u tools/ab_inflate.py --records $N $L > gpurun_out/${T}_ab.log 2>&1
echo "ab rc=$?"
