#!/bin/bash
# scripts/gpu_attrib.sh -- per-phase attribution of both K1 variants on one box
# (the diagnostic build's MIJ_K1_FLAGS removal runs and MIJ_K1_WTIME phase
# clocks, the product build's pattern floor in the same call).  Output:
# gpurun_out/attrib/*.log and a summary on stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/attrib
D=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so
run() {  # tag mode flags [env]
  local tag=$1 mode=$2 flags=$3; shift 3
  env "$@" MIJ_LIB=$D MIJ_K1_FLAGS=$flags timeout -k 10 300 python3 bench.py --mode $mode --steps 10 --warmup 3 \
      --no-cpu-baseline --verify 0 --coef-launches 0 > gpurun_out/attrib/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/attrib/$tag.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/attrib/$tag.log').read().splitlines() if l.startswith('{')][-1]);print('$tag', '$mode', 'flags=$flags', d['stages_ms']['k1_colour_dct_quant'], 'fixups', d.get('fp64_fixups_per_frame'))"
  grep "K1 phases" gpurun_out/attrib/$tag.log || true
}
# product build: the coefficient K1 and its pattern floor (bench's own line)
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 > gpurun_out/attrib/product.log 2>&1 || { echo product failed; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/attrib/product.log').read().strip().splitlines()[-1]);r=d['roofline_k1_coefficient_variant'];print('product token K1', d['stages_ms']['k1_colour_dct_quant'], 'coef K1', r['ms_per_launch'], 'floor', r['pattern_floor_ms'])"
for spec in "c0 dct 0" "c_lut dct 1" "c_rep dct 2" "c_col dct 4" "c_quant dct 32" "c_mfma dct 64" "c_store dct 16" "c_core dct 100" \
            "t0 encode 0" "t_col encode 4" "t_quant encode 32" "t_mfma encode 64" "t_emit encode 4096" "t_acloop encode 8192" \
            "t_hist encode 512" "t_tokst encode 1024" "t_rep encode 2"; do
  run $spec || exit 1
done
run c_wt dct 0 MIJ_K1_WTIME=1 || exit 1
run t_wt encode 0 MIJ_K1_WTIME=1 || exit 1
