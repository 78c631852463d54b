set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/lk_probe.py > gpurun_out/r05d_probe.json 2>&1; cat gpurun_out/r05d_probe.json
DRAM="main" WORK=syn4 STEPS=1000 bash scripts/gpu_ab_session.sh r05d || exit $?
TCI_LIB=$PWD/build/ab/libtci_adaptprof.so timeout -k 10 300 python scripts/synth_dram_time.py 4 1000 > gpurun_out/r05d_adaptprof.json 2> gpurun_out/r05d_adaptprof.err; cat gpurun_out/r05d_adaptprof.json; grep cycles gpurun_out/r05d_adaptprof.err
