set -o pipefail
cd $GRAFT_REPO_ROOT
AB_ARGS="--stream 0 --modes dense,dense16" bash scripts/ab_time.sh lanecnt ablibs/base/libpm.so ablibs/lanecnt/libpm.so || exit 1
