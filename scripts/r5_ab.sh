# Round-5 A/B of general-kernel builds on the from-init windows: C3 / C3-spec first launches
# (1,048,576 clusters), C4-N9 first launches (16,384), c2_init (65,536); per-launch tick-kernel ms.
# Usage: bash scripts/r5_ab.sh TAG LIB [LIB ...]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; T=$1; shift
O=gpurun_out/ab_$T.txt; : > $O
for lib in "$@"; do
  for wl in "c3 1048576 2" "c3_spec 1048576 2" "c4_n9 16384 5" "c4_spec 16384 3" "c2_init 65536 1"; do
    set -- $wl
    echo "== $(basename $lib) $1" >> $O
    timeout -k 10 120 python3 scripts/first_launch.py $1 $2 $3 $lib >> $O 2>&1 || { echo "failed: $lib $wl"; tail -5 $O; exit 1; }
  done
done
cat $O
