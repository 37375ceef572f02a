# round 6: the Kademlia snapshot build at 2^24 (tools/diag/kad_build_time.py): kernel trace, then
# separate PMC passes (SQ, FETCH_SIZE, WRITE_SIZE) per MI355X_MICROARCH.md, summarised per kernel.
# usage: bash tools/gpu_r06_build.sh <outdir> [pmc]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
CMD="python3 tools/diag/kad_build_time.py --reps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $CMD > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
grep '^{' $O/kt.log
if [ "$2" = pmc ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $O/sq -o run -- $CMD > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- $CMD > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- $CMD > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
fi
python3 tools/prof_summary.py $O k_kad_ > $O/summary.txt
rm -rf $O/kt $O/sq $O/fetch $O/write
head -12 $O/summary.txt | cut -c1-200
