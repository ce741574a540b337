cd /root/repo; export TMPDIR=/tmp; mkdir -p gpurun_out/clk
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-include-regex mcu --output-format csv -d gpurun_out/clk/p -o run -- python3 bench.py --mode dct --steps 2 --warmup 1 --no-cpu-baseline --verify 0 > gpurun_out/clk/log 2>&1
