#!/bin/bash
# HPatches-like e2e stream under a kernel + HIP runtime trace: the cold start and the steady-state device gaps
set -o pipefail
mkdir -p gpurun_out/r14d
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $PWD/gpurun_out/r14d/prof -o run -- python3 tools/extract_e2e.py --sizes hpatches --seqs 96 --no-write > gpurun_out/r14d/e2e.txt 2>&1 || { tail -20 gpurun_out/r14d/e2e.txt; exit 1; }
tail -1 gpurun_out/r14d/e2e.txt | cut -c1-300
find $PWD/gpurun_out/r14d/prof -name "*.csv" | xargs ls -la
python3 tools/trace_gaps.py $PWD/gpurun_out/r14d/prof --gap 200 --long 500 --bin 50 > gpurun_out/r14d/gaps.txt 2>&1 || { tail gpurun_out/r14d/gaps.txt; exit 1; }
head -60 gpurun_out/r14d/gaps.txt
tar czf gpurun_out/r14d/prof.tgz -C gpurun_out/r14d prof && rm -rf gpurun_out/r14d/prof
ls -la gpurun_out/r14d
