#!/bin/bash
# scripts/gpu_measure.sh [sections...] -- the measurement runs of a round in
# one GPU call, each under its own time limit, results under gpurun_out/meas/.
#   bench    default bench line (config 3, every slot verified)
#   attrib   K1 time attribution with the diagnostic build's switches
#   c4       config 4 at N=1, root and distributed emission
#   stream   host-fed PPM stream (files -> .jpg, PCIe ceiling)
#   q        the quality sweep (Q=75, Q=90)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/meas; mkdir -p $out
export TMPDIR=/tmp
run() {  # name seconds args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python3 bench.py "$@" > $out/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $out/$name.log; exit 1; }
  grep '^{' $out/$name.log | tail -1 > $out/$name.json
  python3 - "$name" "$out/$name.json" <<'P'
import json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], d.get("ms_per_step"), d.get("value"), d.get("stages_ms") or d.get("phases_ms") or d.get("stage_s_per_step"),
      "verified", d.get("verified_frames", d.get("verified_files")))
P
}
for sec in "${@:-bench}"; do
  case $sec in
    bench) run bench 420 ;;
    attrib)
      [ -f jpeg-encoder-decoder_amd/libmijpeg_diag.so ] || { echo "no diag build"; exit 1; }
      for f in ${FLAGS:-0 1 4 8192 4096}; do
        MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so MIJ_K1_FLAGS=$f \
          run attrib_$f 300 --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --coef-launches 0
      done ;;
    c4)
      run c4_root 300 --workload config4 --steps 20 --warmup 3 --band-emit root
      run c4_bands 300 --workload config4 --steps 20 --warmup 3 --band-emit bands ;;
    stream) run stream 600 --workload stream --steps 3 --warmup 1 ;;
    q)
      run q75 300 --quality 75 --no-cpu-baseline --coef-launches 0
      run q90 300 --quality 90 --no-cpu-baseline --coef-launches 0 ;;
    *) echo "unknown section $sec"; exit 2 ;;
  esac
done
