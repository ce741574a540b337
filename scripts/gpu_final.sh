#!/bin/bash
# closing measurements of a round into gpurun_out/final_<tag> (scripts/gpu_final.sh <tag>):
# default bench (twice), Q sweep, single 1920x1280 frame, config 4 N=1 with the
# root's and the distributed emission (every frame verified), the host-fed
# stream, and the memory-floor probe of K1's access pattern
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/final_${1:-r04}; mkdir -p $out
export TMPDIR=/tmp
run() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs python3 bench.py "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; exit 1; }
  grep '^{' $out/$name.log | tail -1 > $out/$name.json
  python3 -c "import json,sys;d=json.load(open('$out/$name.json'));print(sys.argv[1], d['ms_per_step'], d['value'], d.get('stages_ms') or d.get('phases_ms'), d.get('verified_frames', d.get('verified_files')))" $name
}
for sec in ${SECTIONS:-bench q single c4 stream probe}; do
  case $sec in
    bench) run bench_a 420; run bench_b 300 --no-cpu-baseline ;;
    q) run q75 300 --quality 75 --no-cpu-baseline --coef-launches 0
       run q90 300 --quality 90 --no-cpu-baseline --coef-launches 0 ;;
    single) run single 300 --frames 1 --width 1920 --height 1280 --steps 200 --warmup 20 --no-cpu-baseline --coef-launches 0 ;;
    c4) run c4_root 300 --workload config4 --steps 20 --warmup 3 --band-emit root --verify -1
        run c4_bands 300 --workload config4 --steps 20 --warmup 3 --band-emit bands --verify -1 ;;
    stream) run stream 600 --workload stream --steps 8 --warmup 2 ;;
    probe) timeout -k 10 300 scripts/micro/tile_stream > $out/tile_stream.txt 2>&1 || { echo "probe failed"; tail -5 $out/tile_stream.txt; exit 1; }
           cat $out/tile_stream.txt ;;
  esac
done
