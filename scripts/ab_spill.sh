# A/B of the spill-region cap (old = 8 B/position regions; cNN = NN chunks per wave)
set -o pipefail
cd $GRAFT_REPO_ROOT
for st in 2 3; do AB_ARGS="--stream $st --modes dense,count" bash scripts/ab_time.sh spillcap_s$st ablibs/old/libpm.so ablibs/c32/libpm.so ablibs/c64/libpm.so ablibs/c128/libpm.so || exit 1; done
