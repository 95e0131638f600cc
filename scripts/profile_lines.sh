#!/bin/bash
# rocprofv3 passes over every bench line's workload (GPU box): the headline with every counter group, the other lines
# with the kernel trace and the request-counter pass (fabric bytes, scripts/summarize_profile.py). Output
# gpurun_out/prof_<name>/. Usage: bash scripts/profile_lines.sh [name ...] (default: all)
cd "$GRAFT_REPO_ROOT"
declare -A ARGS=(
  [cfg2]="--config 2"
  [local]="--config 2 --mode local"
  [k31]="--config 3"
  [k70local]="--config 2 --k 70 --mode local"
  [k70err05]="--config 2 --k 70 --mode local --err 0.005"
  [varq]="--config 2 --mode local --qual variable"
  [cfg5]="--config 5 --reads 4000000"
  [cfg5local]="--config 5 --reads 4000000 --mode local"
)
NAMES=${*:-"cfg2 local k31 k70local k70err05 varq cfg5 cfg5local"}
for n in $NAMES; do
  rm -rf gpurun_out/prof_$n
  if [ $n = cfg2 ]; then P="trace req fetch write tcc sq sq2 ta"; else P="trace req tcc"; fi
  PASSES="$P" OUT=gpurun_out/prof_$n bash scripts/profile.sh ${ARGS[$n]} 2> gpurun_out/profile_$n.err || { echo "profile $n failed"; exit 1; }
  echo "profiled $n"
done
echo PROFILES_OK
