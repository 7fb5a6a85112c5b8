# round 5: full GPU suite + smoke on the F(6x6) build
set -o pipefail
mkdir -p gpurun_out/r13q
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r13q/tests.txt 2>&1 || { tail -40 gpurun_out/r13q/tests.txt; exit 1; }
tail -3 gpurun_out/r13q/tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
POSFEAT_HIP_LIB=$PWD/posfeat_amd/libposfeat_hip_ab.so POSFEAT_WINO6=0 POSFEAT_WINO6_ENC=0 timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
