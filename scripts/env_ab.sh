# A/B an env switch on any python micro-bench: bash scripts/env_ab.sh TAG VAR "v0 v1" <python args...>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2; VALS=$3; shift 3
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python "$@" > gpurun_out/${TAG}_${v}.log 2>&1 || exit 1
done
