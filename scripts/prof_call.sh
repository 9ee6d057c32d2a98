# gpurun wrappers: bash scripts/prof_call.sh TAG "WORKLOADS" (scripts/profile_all.sh from the box repo root)
cd $GRAFT_REPO_ROOT && bash scripts/profile_all.sh $1 "$2"
