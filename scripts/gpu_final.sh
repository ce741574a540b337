#!/bin/bash
# closing measurements of a round into gpurun_out/final_<tag> (scripts/gpu_final.sh <tag>):
# default bench (twice), Q sweep, single 1920x1280 frame, config 4 N=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/final_${1:-r04}; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; exit 1; }; tail -1 $out/$name.log > $out/$name.json; python3 -c "import json,sys;d=json.load(open('$out/$name.json'));print(sys.argv[1], d['ms_per_step'], d['value'], d.get('stages_ms'), d.get('verified_frames'))" $name; }
run bench_a
run bench_b --no-cpu-baseline
run q75 --quality 75 --no-cpu-baseline --coef-launches 0
run q90 --quality 90 --no-cpu-baseline --coef-launches 0
run single --frames 1 --width 1920 --height 1280 --steps 200 --warmup 20 --no-cpu-baseline --coef-launches 0
run c4 --workload config4 --steps 20 --warmup 3
