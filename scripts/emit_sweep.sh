cd "${GRAFT_REPO_ROOT:-.}"
for q in 50 90; do
 for s in 16 32 48 96 192 384; do
  timeout -k 10 300 python3 bench.py --quality $q --steps 10 --warmup 3 --no-cpu-baseline --verify 0 --coef-launches 0 --opt emit_slots=$s > gpurun_out/es.log 2>&1 || { tail -3 gpurun_out/es.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/es.log').read().splitlines() if l.startswith('{')][-1]);s=d['stages_ms'];print('Q',sys.argv[1],'slots',sys.argv[2],d['ms_per_step'],'emit',s['emit'],'pack',s['pack'])" $q $s
 done
done
