set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
timeout -k 10 300 python -u tools/diag/k1_sorted.py all 5 > $O/k1sort.json 2> $O/k1sort.err || { tail -20 $O/k1sort.err; exit 1; }
cat $O/k1sort.json
for md in plain presorted; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$md/fetch -o run -- python3 tools/diag/k1_sorted.py $md 3 > $O/f_$md.log 2>&1 || { tail -5 $O/f_$md.log; exit 1; }
  python3 tools/prof_summary.py $O/f_$md k_chord_lanes > $O/f_$md.txt 2>&1 || true
  cat $O/f_$md.txt
  rm -rf $O/f_$md
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_koorde.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/koorde.log 2>&1 || { tail -30 $O/koorde.log; exit 1; }
tail -2 $O/koorde.log
timeout -k 10 300 python -u bench.py --workload K --no-cpu-baseline > $O/bench_K.json 2> $O/bench_K.err || { tail -20 $O/bench_K.err; exit 1; }
cat $O/bench_K.json
bash tools/profile.sh K $O/profK k_koorde_route > $O/profK.log 2>&1 || { tail -20 $O/profK.log; exit 1; }
cat $O/profK/summary.txt | grep -v "^void at::\|rocprim\|rocclr" | head -30
