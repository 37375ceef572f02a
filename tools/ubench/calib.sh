# FETCH_SIZE calibration for random 64 B line gathers (known byte count), one PMC pass per mode.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/tools/ubench
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
for m in 0 2; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/calib$m -o run -- ./gather 16384 $m 100 4 > $O/calib$m.log 2>&1 || exit 1
  python3 - $O/calib$m/run_results.db <<'PY' >> $O/calib.txt
import sqlite3,sys,glob
dbs=glob.glob(sys.argv[1]) or glob.glob(sys.argv[1].replace('run_results.db','*/*.db'))
c=sqlite3.connect(dbs[0])
for name,v,cnt in c.execute("select k.name, sum(e.counter_value), count(distinct e.dispatch_id) from pmc_events e join kernels k on k.dispatch_id=e.dispatch_id where e.counter_name='FETCH_SIZE' group by k.name"):
    print(name[:60], 'FETCH_SIZE KB total', v, 'dispatches', cnt)
PY
  grep table $O/calib$m.log >> $O/calib.txt
done
rm -rf $O/calib0 $O/calib2
cat $O/calib.txt
