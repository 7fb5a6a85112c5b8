# round 5: HPatches-size stream, per-group launch trace and pipeline-depth variants
set -o pipefail
mkdir -p gpurun_out/r13x
export PYTHONUNBUFFERED=1
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u tools/extract_e2e.py --sizes hpatches --seqs 96 > gpurun_out/r13x/e2e_$tag.txt 2>&1 || { tail -20 gpurun_out/r13x/e2e_$tag.txt; return 1; }
  tail -1 gpurun_out/r13x/e2e_$tag.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cold']; print('$tag', round(c['images_per_s'],1), 'replay', round(c['kernel_path_replay_images_per_s'],1), c['host'])"
}
run trace POSFEAT_EXTRACT_TRACE=1 || exit 1
run inf2 POSFEAT_EXTRACT_INFLIGHT=2 || exit 1
run ahead4 POSFEAT_EXTRACT_AHEAD=4 || exit 1
run base || exit 1
