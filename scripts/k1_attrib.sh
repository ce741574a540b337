#!/bin/bash
# scripts/k1_attrib.sh -- K1 time attribution with the diagnostic switches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
[ -f jpeg-encoder-decoder_amd/libmijpeg_diag.so ] || { echo "build it first: make -C jpeg-encoder-decoder_amd diag"; exit 1; }
mkdir -p gpurun_out
for f in ${FLAGS:-0 1 2 3}; do
  echo "flags=$f"
  MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so MIJ_K1_FLAGS=$f timeout -k 10 300 python3 bench.py --mode ${MODE:-encode} ${BENCH_EXTRA:-} --steps 5 --warmup 2 --no-cpu-baseline --verify 0 > gpurun_out/attrib_$f.log 2>&1 || { echo "failed rc=$?"; tail -5 gpurun_out/attrib_$f.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/attrib_$f.log').read().strip().splitlines()[-1]);print(d['stages_ms']['k1_colour_dct_quant'], d.get('fp64_fixups_per_frame'))"
done
