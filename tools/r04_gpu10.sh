set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in s1_prio s2_pool; do
RTG_LIB=$PWD/raytracingrenderer_amd/lib/ab/$v.so timeout -k 10 100 python -u tools/r04_churn.py 300 > gpurun_out/r04_churn_$v.log 2>&1
echo "$v rc $?" >> gpurun_out/r04_churn_$v.log
done
