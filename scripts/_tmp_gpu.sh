bash scripts/gpu_dram_check.sh dr10 || exit 1
TCI_LIB=build/ab/libtci_adaptprof.so timeout -k 10 60 python scripts/dram_time.py 20000 fused 20
VARIANTS="ship" bash scripts/gpu_dram_ab.sh dab10 20000
