set -e
mkdir -p gpurun_out
timeout -k 10 120 python scripts/dram_time.py 20000 fused > gpurun_out/dt_ship.json 2> gpurun_out/dt_ship.err
TCI_LIB=build/ab/libtci_chainprof.so timeout -k 10 120 python scripts/dram_time.py 20000 fused > gpurun_out/dt_prof.json 2> gpurun_out/dt_prof.err
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dt_rp -o trace -- python3 scripts/dram_time.py 20000 fused > gpurun_out/dt_rp.json 2> gpurun_out/dt_rp.err
cat gpurun_out/dt_ship.json gpurun_out/dt_prof.json; tail -2 gpurun_out/dt_prof.err
