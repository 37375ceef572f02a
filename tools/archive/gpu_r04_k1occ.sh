# round-4: K1 at 5 waves/SIMD in every instantiation (the shard step had 4) -- A/B against the
# old bounds (-DOVS_K1_WAVES=1) on the W = 8 emulation of config C, single C and sharded C at W = 1;
# SQ counters of the W = 8 emulation; Chord shard parity suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export OVS_SKIP_BUILD=1
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29631
[ "$2" = notests ] || timeout -k 10 600 python -u -m pytest tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
[ "$2" = notests ] || tail -1 $O/tests.log
for tag in main k1w1; do
  if [ $tag = main ]; then unset OVS_LIB; else export OVS_LIB=$PWD/oversim_amd/libovs_kbr_$tag.so; fi
  timeout -k 10 300 python -u tools/diag/shard_w8_model.py --workload C > $O/w8_C_$tag.jsonl 2> $O/w8_C_$tag.err || { tail -20 $O/w8_C_$tag.err; exit 1; }
  echo "$tag $(tail -1 $O/w8_C_$tag.jsonl | cut -c1-400)"
  for rep in 1 2; do
    timeout -k 10 300 python -u bench.py --workload C --no-cpu-baseline > $O/bench_C_${tag}_$rep.json 2> $O/bench_C_${tag}_$rep.err || { tail -20 $O/bench_C_${tag}_$rep.err; exit 1; }
    OVS_BENCH_SHARD=1 timeout -k 10 300 python -u bench.py --workload C --no-cpu-baseline > $O/bench_Cshard_${tag}_$rep.json 2> $O/bench_Cshard_${tag}_$rep.err || { tail -20 $O/bench_Cshard_${tag}_$rep.err; exit 1; }
    python -c "import json,sys; a=json.load(open(sys.argv[1])); b=json.load(open(sys.argv[2])); print(sys.argv[3], 'C single %.3f ms  C shard W=1 %.3f ms' % (a['ms_per_step'], b['ms_per_step']))" $O/bench_C_${tag}_$rep.json $O/bench_Cshard_${tag}_$rep.json $tag
  done
done
unset OVS_LIB
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $O/pmc/sq -o run -- python3 tools/diag/shard_w8_model.py --workload C > $O/pmc_sq.log 2>&1 || { tail -5 $O/pmc_sq.log; exit 1; }
python tools/prof_summary.py $O/pmc k_chord_lanes > $O/pmc_sq.txt && rm -rf $O/pmc
grep SQ_ $O/pmc_sq.txt | head -8
