set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export OVS_SKIP_BUILD=1
O=gpurun_out/r04_f_k2ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kad.py tests/test_gpu_timed.py -m gpu -x -q --timeout 300 --timeout-method thread -k "kad or Kad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab.sh r04_f_k2ab "E B" old w4 preg
