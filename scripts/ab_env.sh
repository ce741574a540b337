cd "${GRAFT_REPO_ROOT}"
for r in 1 2; do
for v in "cur:" "cur:MIJ_PACK_SPLIT=1" "m4kns:"; do
  lib=${v%%:*}; ev=${v#*:}
  env $ev MIJ_LIB=$PWD/ab/libmijpeg_$lib.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 > gpurun_out/ab.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);s=d['stages_ms'];print(sys.argv[1], round(d['ms_per_step'],3), 'k1', s['k1_colour_dct_quant'], 'pack', s.get('pack'), 'emit', s.get('emit'))" "$v"
done; done
