# Kernel-trace breakdown of one bench.py configuration: NAME=<tag> bash scripts/_gpu_prof_bench.sh <bench args>
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/prof
mkdir -p $O
N=${NAME:-run}
timeout -k 10 480 rocprofv3 --kernel-trace -d $O/db_$N -o run -- python3 bench.py "$@" > $O/$N.log 2>&1 || { tail -20 $O/$N.log; exit 1; }
DB=$(find $O/db_$N -name "*results.db" | head -1)
python tools/rocpd_summary.py $DB --steps ${PSTEPS:-2} --csv $O/kernels_$N.csv > $O/breakdown_$N.txt
head -30 $O/breakdown_$N.txt
if [ "${OVERLAP:-0}" = "1" ]; then python tools/trace_overlap.py $DB --steps ${PSTEPS:-2} > $O/overlap_$N.txt; head -40 $O/overlap_$N.txt; fi
rm -rf $O/db_$N
