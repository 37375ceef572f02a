#!/bin/bash
# Build the compaction micro-benchmark (tools/diag/compact_bench.hip, the in-tree compact.hip) into
# tools/diag/_cbench/; `tools/diag/compact_bench.sh run` runs it (GPU).
set -e
cd "$(dirname "$0")/../.."
D=tools/diag/_cbench; mkdir -p $D
if [ "${1:-}" = run ]; then
  timeout -k 5 60 $D/cb
  exit 0
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -w -I include -x hip tools/diag/compact_bench.hip -o $D/cb
